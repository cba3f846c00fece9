// Rollout-side kernels of the fused on-policy pipeline (gfx950):
//   K4 xpa_gather_minibatch  minibatch row gather + advantage moments (memory_tools.py:231-242)
//   K5 xpa_rms_*             RunningMeanStd + obs normalisation (statistic_tools.py:63-112, agent.py:104-116)
//   K3 xpa_rollout_sample    action sample + log-prob + buffer store (ppoclip_agent.py:50-57, memory_tools.py:196-204)
//   K7 xpa_synthbox_step     synthetic env step with auto-reset (gym_vec_env.py:201-212 contract)
//   K8 xpa_rollout_post      reward norm, return tracker, ret_rms, path closures (ppoclip_agent.py:68-101)
// All per-step kernels read the buffer column from a device cursor so a whole env step can be
// captured once in a hipGraph and replayed.
#include "cartpole_body.h"

namespace {

constexpr int kGatherRows = 64;  // rows per gather block == rows per adv partial (1024 blocks at B = 65 536)
constexpr int kRmsRows = 256;     // rows per RMS partial block
// threads per RMS partial block: 1024 for wide observations (r02: with 256, C4's 376 columns had one thread per column
// walking all 256 rows, 43.8 us per env step -> 17.9 us), 256 for narrow ones (C1 / C2: the reduction and the merge
// stay as short as before)
constexpr int kRmsWideDim = 64;
constexpr uint32_t kSaltAct = 0xAC7105EDu;
constexpr uint32_t kSaltReset = 0x5EED0000u;  // oracle/synth_env.py SALT_RESET

// ---------------------------------------------------------------------------------------------
// K4 gather
// ---------------------------------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(256) void gather_rows_kernel(const int64_t *__restrict__ idx, int64_t batch,
                                                          int64_t n_rows, const V *__restrict__ src, int64_t row_vecs,
                                                          V *__restrict__ dst, const float *__restrict__ adv,
                                                          double *__restrict__ adv_partials, int *__restrict__ err,
                                                          int64_t out_vecs = -1) {
    __shared__ double s_red[4];
    __shared__ int64_t s_src[kGatherRows];
    const int64_t r0 = (int64_t)blockIdx.x * kGatherRows;
    const int64_t r1 = r0 + kGatherRows < batch ? r0 + kGatherRows : batch;
    const int nr = (int)(r1 - r0);
    if ((int)threadIdx.x < nr) {
        const int64_t sr = idx[r0 + threadIdx.x];
        s_src[threadIdx.x] = sr;
        if (err && (sr < 0 || sr >= n_rows)) atomicAdd(err, 1);  // the row is zero-filled, and counted
    }
    __syncthreads();
    // Consecutive lanes copy consecutive vectors of a row (32-bit index math; the row's source offset
    // comes from LDS), so each row is one contiguous burst.
    // out_vecs (r05): the output row pitch in vectors (-1: packed rows); the pitch's tail of each row is not written
    const uint32_t rv = (uint32_t)row_vecs;
    const uint32_t n = (uint32_t)nr * rv;
    const int64_t op = out_vecs < 0 ? row_vecs : out_vecs;
    V *out = dst + r0 * op;
    for (uint32_t e = threadIdx.x; e < n; e += 256) {
        const uint32_t r = e / rv;
        const uint32_t c = e - r * rv;
        const int64_t sr = s_src[r];
        out[(int64_t)r * op + c] = (sr >= 0 && sr < n_rows) ? src[sr * row_vecs + c] : V{};
    }
    if (adv_partials) {
        double s = 0.0, q = 0.0;
        const int64_t sr = (int)threadIdx.x < nr ? s_src[threadIdx.x] : -1;
        if (sr >= 0 && sr < n_rows) {
            const double a = (double)adv[sr];
            s = a;
            q = a * a;
        }
        s = xpa_block_sum(s, s_red, 4);
        q = xpa_block_sum(q, s_red, 4);
        if (threadIdx.x == 0) {
            adv_partials[2 * blockIdx.x] = s;
            adv_partials[2 * blockIdx.x + 1] = q;
        }
    }
}

// Wide rows (>= 4 KiB, e.g. 4x84x84 uint8 frames of the replay buffer): one block per (row, 16 KiB
// chunk), four independent 16-B non-temporal loads per thread in flight.
constexpr int kWideU = 4;
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void gather_wide_kernel(const int64_t *__restrict__ idx, int64_t n_rows,
                                                          const u4v *__restrict__ src, int64_t row_vecs,
                                                          int64_t chunks, u4v *__restrict__ dst, int *__restrict__ err) {
    const int64_t row = (int64_t)blockIdx.x / chunks, chunk = (int64_t)blockIdx.x - row * chunks;
    const int64_t sr = idx[row];
    const bool ok = sr >= 0 && sr < n_rows;
    if (err && !ok && chunk == 0 && threadIdx.x == 0) atomicAdd(err, 1);
    const int64_t c0 = chunk * 256 * kWideU + threadIdx.x;
    u4v v[kWideU];
#pragma unroll
    for (int u = 0; u < kWideU; ++u) {
        const int64_t c = c0 + u * 256;
        v[u] = (ok && c < row_vecs) ? __builtin_nontemporal_load(src + sr * row_vecs + c) : u4v{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < kWideU; ++u) {
        const int64_t c = c0 + u * 256;
        if (c < row_vecs) __builtin_nontemporal_store(v[u], dst + row * row_vecs + c);
    }
}

// Column store: dst[(n * horizon + cursor->ptr) * row_vecs + c] = src[n * row_vecs + c] (raw uint8
// Atari observations into the rollout buffer, DummyOnPolicyBuffer_Atari.store, memory_tools.py:196-204).
__global__ __launch_bounds__(256) void store_column_kernel(const u4v *__restrict__ src, int64_t n, int64_t row_vecs,
                                                           u4v *__restrict__ dst, int64_t horizon,
                                                           const xpa_cursor_t *__restrict__ cur) {
    const int64_t t = cur->ptr;
    const int64_t total = n * row_vecs;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t r = e / row_vecs, c = e - r * row_vecs;
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + e), dst + (r * horizon + t) * row_vecs + c);
    }
}

// Epoch permutation of [0, n) (the np.random.shuffle of ppoclip_agent.py:76-81): a 4-round Feistel
// network over 2h bits (2^(2h) >= n) keyed by a counter hash of (seed, counter), cycle-walked into
// [0, n) — a bijection computed independently per element, one launch, no sort.
constexpr uint32_t kSaltPerm = 0x9E2A0000u;
__device__ __forceinline__ uint32_t feistel(uint32_t x, int h, uint32_t seed, uint32_t counter) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t L = x >> h, R = x & mask;
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t F = xpa_hash4(seed ^ kSaltPerm, counter, r, R) & mask;
        const uint32_t nl = R;
        R = L ^ F;
        L = nl;
    }
    return (L << h) | R;
}

__global__ __launch_bounds__(256) void permutation_kernel(int64_t n, int h, uint32_t seed, uint32_t counter,
                                                          int64_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t x = (uint32_t)i;
    do {
        x = feistel(x, h, seed, counter);
    } while ((int64_t)x >= n);
    out[i] = (int64_t)x;
}

// ---------------------------------------------------------------------------------------------
// K5 RunningMeanStd
// ---------------------------------------------------------------------------------------------
// Block g sums rows [g*kRmsRows, (g+1)*kRmsRows) of (x - shift) and (x - shift)^2 in f64 per column
// (shift = the running mean, so the one-pass variance does not cancel).  Threads cover a
// (row group x column) tile, all row loads of a thread are independent (no serial latency chain),
// and the row groups are combined through LDS in a fixed order.
__device__ void rms_merge_body(const double *part, int64_t np, int64_t n, int64_t dim, float *__restrict__ mean,
                               float *__restrict__ var, double *__restrict__ count);

// MERGE: the last block to finish (atomic ticket) also runs the merge below over all blocks' partials in
// block order (deterministic, = xpa_rms_merge) and resets the ticket: one launch per obs-RMS update.
template <bool MERGE, int kRmsThreads>
__global__ __launch_bounds__(kRmsThreads) void rms_partials_kernel(const float *__restrict__ x, int64_t n, int64_t dim,
                                                                   int64_t ld, const float *shift,  // may alias mean
                                                                   double *__restrict__ part, float *mean,
                                                                   float *__restrict__ var, double *__restrict__ count,
                                                                   unsigned int *__restrict__ ticket) {
    __shared__ double s_sum[kRmsThreads], s_sq[kRmsThreads];
    __shared__ bool s_last;
    const int64_t r0 = (int64_t)blockIdx.x * kRmsRows;
    const int64_t r1 = r0 + kRmsRows < n ? r0 + kRmsRows : n;
    const int64_t np = gridDim.x;
    for (int64_t c0 = 0; c0 < dim; c0 += 256) {
        const int dc = (int)(dim - c0 < 256 ? dim - c0 : 256);  // columns in this tile
        const int groups = kRmsThreads / dc;                    // row groups
        const int c = threadIdx.x % dc, gsub = threadIdx.x / dc;
        double s = 0.0, q = 0.0;
        if (gsub < groups) {
            const float sh = shift ? shift[c0 + c] : 0.f;
            // 16 rows' loads issued before their (in-order) accumulation: one memory round trip per 16 rows (the
            // unroll-4 loop waited once per 4 rows: ~5 serial HBM round trips per thread at C2's 17 columns)
            for (int64_t rb = r0 + gsub; rb < r1; rb += 16 * (int64_t)groups) {
                float xv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t r = rb + (int64_t)u * groups;
                    xv[u] = x[(r < r1 ? r : rb) * ld + c0 + c];
                }
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (rb + (int64_t)u * groups < r1) {
                        const double v = (double)xv[u] - (double)sh;
                        s += v;
                        q += v * v;
                    }
            }
        }
        s_sum[threadIdx.x] = s;
        s_sq[threadIdx.x] = q;
        __syncthreads();
        if ((int)threadIdx.x < dc) {
            double ts = 0.0, tq = 0.0;
            for (int k = 0; k < groups; ++k) {
                ts += s_sum[k * dc + threadIdx.x];
                tq += s_sq[k * dc + threadIdx.x];
            }
            xpa_store_agent(part + (int64_t)blockIdx.x * dim + c0 + threadIdx.x, ts);  // sc1: handed to the
            xpa_store_agent(part + (np + blockIdx.x) * dim + c0 + threadIdx.x, tq);    // merging block
        }
        __syncthreads();
    }
    if (MERGE) {
        xpa_drain();
        __syncthreads();
        if (threadIdx.x == 0) s_last = xpa_ticket(ticket) == (unsigned)(np - 1);
        __syncthreads();
        if (!s_last) return;
        rms_merge_body(part, np, n, dim, mean, var, count);
        if (threadIdx.x == 0) *ticket = 0u;
    }
}

// r05, wide observations (dim > kRmsWideDim, C4's 376): the same partials from a 2-D grid — block (g, cb) takes row
// block g (kRmsRows rows) x columns 64 cb .. + 63, thread (group j, column c) sums rows j, j + 16, ... (16 loads in
// flight) and the 16 groups are added in order — so np x ceil(dim / 64) blocks share the chip (the 1-D form ran the
// 16 row blocks of a 4096-env step on 16 CUs: 21.5 us); the last of all the blocks merges (rms_merge_body, np = gridDim.x)
template <bool MERGE>
__global__ __launch_bounds__(1024) void rms_partials_cols_kernel(const float *__restrict__ x, int64_t n, int64_t dim,
                                                                  int64_t ld, const float *shift,
                                                                  double *__restrict__ part, float *mean,
                                                                  float *__restrict__ var, double *__restrict__ count,
                                                                  unsigned int *__restrict__ ticket) {
    __shared__ double s_sum[16][64], s_sq[16][64];
    __shared__ bool s_last;
    const int64_t r0 = (int64_t)blockIdx.x * kRmsRows;
    const int64_t r1 = r0 + kRmsRows < n ? r0 + kRmsRows : n;
    const int64_t np = gridDim.x;
    const int64_t c0 = (int64_t)blockIdx.y * 64;
    const int c = threadIdx.x & 63, j = threadIdx.x >> 6;
    double s = 0.0, q = 0.0;
    if (c0 + c < dim) {
        const float sh = shift ? shift[c0 + c] : 0.f;
        for (int64_t rb = r0 + j; rb < r1; rb += 16 * 16) {
            float xv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int64_t r = rb + (int64_t)u * 16;
                xv[u] = x[(r < r1 ? r : rb) * ld + c0 + c];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (rb + (int64_t)u * 16 < r1) {
                    const double v = (double)xv[u] - (double)sh;
                    s += v;
                    q += v * v;
                }
        }
    }
    s_sum[j][c] = s;
    s_sq[j][c] = q;
    __syncthreads();
    if (threadIdx.x < 64 && c0 + threadIdx.x < dim) {
        double ts = s_sum[0][threadIdx.x], tq = s_sq[0][threadIdx.x];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            ts += s_sum[k][threadIdx.x];
            tq += s_sq[k][threadIdx.x];
        }
        xpa_store_agent(part + (int64_t)blockIdx.x * dim + c0 + threadIdx.x, ts);
        xpa_store_agent(part + (np + blockIdx.x) * dim + c0 + threadIdx.x, tq);
    }
    if (MERGE) {
        xpa_drain();
        __syncthreads();
        if (threadIdx.x == 0) s_last = xpa_ticket(ticket) == (unsigned)(gridDim.x * gridDim.y - 1);
        __syncthreads();
        if (!s_last) return;
        rms_merge_body(part, np, n, dim, mean, var, count);
        if (threadIdx.x == 0) *ticket = 0u;
    }
}

// Sum of the partials (fixed order) -> batch mean/var, then update_from_moments
// (statistic_tools.py:86-112) into mean/var (f32) and count (f64).  mean doubles as the shift the
// partials were taken around.
// Every (partial, column) sum / square is loaded by its own thread into LDS in one round trip (sc1 loads:
// the partials may come from other blocks of the same launch), then each column is summed over the
// partials in block order (deterministic).
constexpr int kMergeLds = 2048;  // doubles of LDS staging: np * dim <= 1024 (else per-column global loads)
// column d of the merge: s / q = the batch's sums of (x - mean[d]) and its square over n rows, c0 = the running count
__device__ __forceinline__ void rms_merge_col(double s, double q, double n, double c0, float *mean, float *var,
                                              int64_t d) {
    const double ms = s / n;
    const double m0 = (double)mean[d], v0 = (double)var[d];
    const double bm = m0 + ms;                        // batch mean
    const double bvar = fmax(q / n - ms * ms, 0.0);   // np.std(x, axis=0)**2 (ddof 0)
    const double tot = c0 + n;
    const double delta = bm - m0;
    const double new_mean = m0 + delta * n / tot;
    const double m2 = v0 * c0 + bvar * n + delta * delta * c0 * n / tot;
    mean[d] = (float)new_mean;
    var[d] = (float)(m2 / tot);
}

__device__ void rms_merge_body(const double *part, int64_t np, int64_t n, int64_t dim, float *__restrict__ mean,
                               float *__restrict__ var, double *__restrict__ count) {
    __shared__ double s_part[kMergeLds];
    const double c0 = *count;
    const bool staged = np * dim * 2 <= kMergeLds;
    if (staged)
        for (int64_t i = threadIdx.x; i < 2 * np * dim; i += blockDim.x) s_part[i] = xpa_load_agent(part + i);
    __syncthreads();
    for (int64_t d = threadIdx.x; d < dim; d += blockDim.x) {
        double s = 0.0, q = 0.0;
        for (int64_t p = 0; p < np; ++p) {
            s += staged ? s_part[p * dim + d] : xpa_load_agent(part + p * dim + d);
            q += staged ? s_part[(np + p) * dim + d] : xpa_load_agent(part + (np + p) * dim + d);
        }
        rms_merge_col(s, q, (double)n, c0, mean, var, d);
    }
    __syncthreads();
    if (threadIdx.x == 0) *count = c0 + (double)n;
}

__global__ __launch_bounds__(256) void rms_merge_kernel(const double *__restrict__ part, int64_t np, int64_t n,
                                                        int64_t dim, float *__restrict__ mean, float *__restrict__ var,
                                                        double *__restrict__ count) {
    rms_merge_body(part, np, n, dim, mean, var, count);
}

__global__ __launch_bounds__(256) void obs_normalize_kernel(const float *__restrict__ x, int64_t n, int64_t dim,
                                                            int64_t ldx, const float *__restrict__ mean,
                                                            const float *__restrict__ var, float clip_range,
                                                            float *__restrict__ out, int64_t ldo,
                                                            float *__restrict__ col_out, int64_t col_ld,
                                                            const xpa_cursor_t *__restrict__ cursor) {
    const int64_t total = n * dim;
    const int64_t coff = (col_out && cursor) ? (int64_t)cursor->ptr * dim : 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / dim, d = e % dim;
        const float sd = sqrtf(var[d]);
        float y = (x[r * ldx + d] - mean[d]) / (sd + 1e-8f);
        y = fminf(fmaxf(y, -clip_range), clip_range);
        out[r * ldo + d] = y;
        if (col_out) col_out[r * col_ld + coff + d] = y;
    }
}

// ---------------------------------------------------------------------------------------------
// K3 sample + log-prob + store
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void gauss_sample_store(int64_t n, int A, int64_t T, const float *mu_row,
                                                   const float *__restrict__ logstd, float v,
                                                   const xpa_cursor_t *__restrict__ cur, uint32_t seed, float act_clip,
                                                   float *__restrict__ buf_act, float *__restrict__ buf_logp,
                                                   float *__restrict__ buf_val, float *__restrict__ env_in,
                                                   int64_t ld_env) {
    const int64_t t = cur->ptr;
    const uint32_t step = cur->step;
    const int64_t cell = n * T + t;
    float logp = 0.f;
    for (int a = 0; a < A; ++a) {
        const uint32_t h1 = xpa_hash4(seed ^ kSaltAct, step, (uint32_t)n, (uint32_t)(2 * a));
        const uint32_t h2 = xpa_hash4(seed ^ kSaltAct, step, (uint32_t)n, (uint32_t)(2 * a + 1));
        const float u1 = 1.0f - xpa_u01(h1);  // (0, 1]
        const float u2 = xpa_u01(h2);
        const float eps = sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
        const float sc = expf(logstd[a]);
        const float m = mu_row[a];
        const float x = m + sc * eps;
        const float diff = x - m;
        logp += -(diff * diff) / (2.0f * sc * sc) - logf(sc) - 0.91893853320467274178f;
        buf_act[cell * A + a] = x;
        env_in[n * ld_env + a] = fminf(fmaxf(x, -act_clip), act_clip);
    }
    buf_logp[cell] = logp;
    buf_val[cell] = v;
}

// Returns the sampled action (K32 steps its env with it).
__device__ __forceinline__ int cat_sample_store_at(int64_t n, int K, int64_t T, int32_t t, uint32_t step,
                                                   const float *z, float v, uint32_t seed, float *__restrict__ buf_act,
                                                   float *__restrict__ buf_logp, float *__restrict__ buf_val,
                                                   float *__restrict__ env_in, int64_t ld_env) {
    const int64_t cell = n * T + t;
    float m = z[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, z[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(z[k] - m);
    const float lse = m + logf(se);
    const float u = xpa_u01(xpa_hash4(seed ^ kSaltAct, step, (uint32_t)n, 0u));
    int pick = K - 1;
    float cdf = 0.f;
    for (int k = 0; k < K; ++k) {
        cdf += expf(z[k] - lse);
        if (u < cdf) {
            pick = k;
            break;
        }
    }
    buf_act[cell] = (float)pick;
    buf_logp[cell] = z[pick] - lse;
    buf_val[cell] = v;
    for (int k = 0; k < K; ++k) env_in[n * ld_env + k] = (k == pick) ? 1.f : 0.f;
    return pick;
}

__device__ __forceinline__ void cat_sample_store(int64_t n, int K, int64_t T, const float *z, float v,
                                                 const xpa_cursor_t *__restrict__ cur, uint32_t seed,
                                                 float *__restrict__ buf_act, float *__restrict__ buf_logp,
                                                 float *__restrict__ buf_val, float *__restrict__ env_in,
                                                 int64_t ld_env) {
    cat_sample_store_at(n, K, T, cur->ptr, cur->step, z, v, seed, buf_act, buf_logp, buf_val, env_in, ld_env);
}

__global__ __launch_bounds__(256) void rollout_sample_gauss_kernel(
    int64_t n_envs, int A, int64_t T, const float *__restrict__ mu, const float *__restrict__ logstd,
    const float *__restrict__ v, const xpa_cursor_t *__restrict__ cur, uint32_t seed, float act_clip,
    float *__restrict__ buf_act, float *__restrict__ buf_logp, float *__restrict__ buf_val, float *__restrict__ env_in,
    int64_t ld_env) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_envs) return;
    gauss_sample_store(n, A, T, mu + n * A, logstd, v[n], cur, seed, act_clip, buf_act, buf_logp, buf_val, env_in,
                       ld_env);
}

__global__ __launch_bounds__(256) void rollout_sample_cat_kernel(
    int64_t n_envs, int K, int64_t T, const float *__restrict__ logits, const float *__restrict__ v,
    const xpa_cursor_t *__restrict__ cur, uint32_t seed, float *__restrict__ buf_act, float *__restrict__ buf_logp,
    float *__restrict__ buf_val, float *__restrict__ env_in, int64_t ld_env) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_envs) return;
    cat_sample_store(n, K, T, logits + n * K, v[n], cur, seed, buf_act, buf_logp, buf_val, env_in, ld_env);
}

// ---------------------------------------------------------------------------------------------
// K14 rollout policy head: hidden activation + output layers (one wave per env, lane l owns hidden
// columns [4l, 4l + 4), butterfly dot products) + the K3 sample/store above, or the value alone.
// ---------------------------------------------------------------------------------------------
// K7's per-env body, shared by the standalone env step and K14's fused form: one wave per env, lanes over
// the state dims; pre(d) = the env's pre-activation for state dim d (row d of [W | U] (s | a)).
struct SynthEnvArgs {
    int D;
    uint32_t seed;
    int max_steps;
    float noise, thresh, reset_scale;
    float *state;
    int64_t ld_state;
    float *final_obs, *rew;
    uint8_t *term, *trunc;
    int32_t *ep_step;
    uint32_t *ep_index;
    float *ep_score, *ep_last_score;
    int32_t *ep_last_len;
    const float *wt;  // fused form: [W | U]^T, [D + A, D] row-major
};

// What K14F's post tail needs from the step, in registers: reward and flags (every lane), and lane d's final observation
// (sv) and next state (sn) for d = lane < min(D, 64)
struct EnvRowOut {
    float r, sv, sn;
    bool te, tr;
};

// t, ep, score0: the env's ep_step / ep_index / ep_score (loaded by the caller, early in the fused form)
template <class PreFn>
__device__ __forceinline__ EnvRowOut synthbox_env_row(int64_t n, int lane, const SynthEnvArgs &e, PreFn pre, int t,
                                                      uint32_t ep, float score0) {
    const int D = e.D;
    EnvRowOut o{0.f, 0.f, 0.f, false, false};
    float sumsq = 0.f, s0 = 0.f;
    for (int d = lane; d < D; d += 64) {
        const uint32_t base = ((uint32_t)t * (uint32_t)D + (uint32_t)d) * 4u;
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += xpa_u01(xpa_hash4(e.seed, (uint32_t)n, ep, base + (uint32_t)j));
        const float xi = (acc - 2.0f) * 1.7320508075688772f;
        const float sv = tanhf(pre(d) + e.noise * xi);
        e.final_obs[n * D + d] = sv;
        sumsq += sv * sv;
        if (d == 0) s0 = sv;
        if (d == lane) o.sv = sv;
    }
    sumsq = xpa_wave_sum(sumsq);
    s0 = __shfl(s0, 0, 64);
    const float r = -sumsq / (float)D;
    const bool te = s0 > e.thresh;
    const int t1 = t + 1;
    const bool tr = t1 >= e.max_steps;
    const bool done = te || tr;
    const float score = score0 + r;
    for (int d = lane; d < D; d += 64) {
        float sn;
        if (done) {
            const uint32_t h = xpa_hash4(e.seed ^ kSaltReset, (uint32_t)n, ep + 1u, (uint32_t)d);
            sn = (2.0f * xpa_u01(h) - 1.0f) * e.reset_scale;
        } else {
            sn = e.final_obs[n * D + d];
        }
        e.state[n * e.ld_state + d] = sn;
        if (d == lane) o.sn = sn;
    }
    o.r = r;
    o.te = te;
    o.tr = tr;
    if (lane == 0) {
        e.rew[n] = r;
        e.term[n] = te ? 1 : 0;
        e.trunc[n] = tr ? 1 : 0;
        if (done) {
            e.ep_last_score[n] = score;
            e.ep_last_len[n] = t1;
            e.ep_index[n] = ep + 1u;
            e.ep_step[n] = 0;
            e.ep_score[n] = 0.f;
        } else {
            e.ep_step[n] = t1;
            e.ep_score[n] = score;
        }
    }
    return o;
}

__device__ __forceinline__ float wave_allsum_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// obs_normalize_kernel's arithmetic on one element (K8's NORM form and K14F)
__device__ __forceinline__ float obs_norm1(float x, float m, float v, float clip) {
    const float sd = sqrtf(v);
    const float y = (x - m) / (sd + 1e-8f);
    return fminf(fmaxf(y, -clip), clip);
}

// ret_rms.update_from_moments (statistic_tools.py:86-112) from the summed (count, sum, sumsq) of the closed paths.
__device__ __forceinline__ void ret_rms_merge_local(double c, double s1, double s2, float &m, float &v, double &cnt) {
    if (c > 0.0) {
        const double bm = s1 / c;
        const double bvar = fmax(s2 / c - bm * bm, 0.0);
        const double c0 = cnt, m0 = (double)m, v0 = (double)v;
        const double tot = c0 + c;
        const double delta = bm - m0;
        m = (float)(m0 + delta * c / tot);
        v = (float)((v0 * c0 + bvar * c + delta * delta * c0 * c / tot) / tot);
        cnt = tot;
    }
}

__device__ __forceinline__ void ret_rms_merge(double c, double s1, double s2, float *ret_mean, float *ret_var,
                                              double *ret_count) {
    if (c > 0.0) {
        float m = *ret_mean, v = *ret_var;
        double cnt = *ret_count;
        ret_rms_merge_local(c, s1, s2, m, v, cnt);
        *ret_mean = m;
        *ret_var = v;
        *ret_count = cnt;
    }
}

// ---- K14F (r06): K8's deferred, normalised post step and the next step's obs_rms.update in K14E's launch ----------------
// An env step of the C2 rollout then takes three launches (normalise + trunk, K40R, K14F) instead of five (+ K8 + K5).
// Per env (one wave, lanes over the state dims) the tail does what post_env<true, true> does for it (reward
// normalisation, buffer column t, closures, kept truncation rows, boot_norm at the last step, the return tracker) from the
// step's results in registers (EnvRowOut) and forms the env's share of the ret_rms moments and of the next observation's
// sums around the running mean; the 4 envs of a block are added in wave order.  The block partials (P = 3 + 2D f64) are
// reduced in two ticketed levels, both in a fixed order (any arrival order gives the same bits): the last block of each
// group of kPostGrp blocks sums its group's partials (4 contiguous chunks, then the chunks in order), and the last group
// to finish sums the group partials in group order, merges obs_rms (rms_merge_col) and ret_rms (ret_rms_merge), advances
// the cursor and resets the tickets.  Every block reads the statistics and the cursor before its ticket, the final block
// writes them after every ticket was taken (K8's protocol).
constexpr int kPostGrp = 64;
// tickets 256 B apart: atomics on one line serialise, and 1024 blocks' tickets on the two lines of a packed [1 + 16]
// array cost ~10 us per launch (tools/k14f_probe.py, r06: drain + group tickets 9.6 us packed)
constexpr int kTicketStride = 64;
// diagnostics (tools/k14f_probe.py, xpa_k14f_probe): bit 1 = the tail ends after the block partial stores, bit 2 = after
// the group tickets, bit 4 = after the group sums (results then invalid: timing only); 0 in production
__device__ int g_k14f_probe = 0;
struct PostArgs {
    xpa_cursor_t *cur;
    float *ret_mean, *ret_var;
    double *ret_count;
    float *returns, *buf_rew, *buf_term;
    uint8_t *buf_closed;
    float *buf_boot;
    float gamma, rew_range, obs_clip;
    int mask_returns, use_rewnorm, atari_lifeloss, slot_from_next, n_slots;
    float *slot_obs;
    int32_t *slot_t, *overflow;
    float *obs_mean, *obs_var;
    double *obs_count;   // nullptr: no obs_rms update (P = 3)
    float *boot_norm;
    int64_t ld_norm;
    double *part;        // f64 [(blocks + groups) * P]
    unsigned *tickets;   // [(1 + groups) * kTicketStride] (ticket i at i * kTicketStride), zero between launches
};

__device__ __forceinline__ void k14f_tail(const PostArgs &pa, int D, const EnvRowOut &eo, bool valid, int64_t n,
                                          int64_t n_envs, int64_t T, int lane, int wave) {
    __shared__ double s_pp[4][3 + 2 * 64];
    __shared__ double s_ch[4][3 + 2 * 64];
    __shared__ bool s_last;
    const bool rms = pa.obs_count != nullptr;
    const int P = 3 + (rms ? 2 * D : 0);
    const int32_t t = pa.cur->ptr;
    double cnt = 0.0, sm = 0.0, sq = 0.0, rp = 0.0, rq = 0.0;
    if (valid) {   // wave-uniform
        const bool last = t == (int32_t)(T - 1);
        const int64_t cell = n * T + t;
        const bool done = eo.te || eo.tr;
        const bool close = last || (done && !(pa.atari_lifeloss && !eo.tr));
        const float m = lane < D ? pa.obs_mean[lane] : 0.f, v = lane < D ? pa.obs_var[lane] : 1.f;
        if (lane == 0) {
            const float rstd = fminf(fmaxf(sqrtf(*pa.ret_var), 0.1f), 100.0f);
            pa.buf_rew[cell] = pa.use_rewnorm ? fminf(fmaxf(eo.r / rstd, -pa.rew_range), pa.rew_range) : eo.r;
            pa.buf_term[cell] = eo.te ? 1.f : 0.f;
            pa.buf_closed[cell] = close ? 1 : 0;
            pa.buf_boot[cell] = 0.f;   // deferred: the bootstraps are written after the rollout
            const float R = pa.returns[n];
            float Rk = pa.mask_returns ? (eo.te ? 0.f : pa.gamma * R) + eo.r : pa.gamma * R + eo.r;
            if (done) {
                cnt = 1.0;
                sm = (double)Rk;
                sq = (double)Rk * (double)Rk;
                Rk = 0.f;
            }
            pa.returns[n] = Rk;
        }
        if (close && !eo.te && !last) {   // mid-buffer truncation: keep the normalised row for later
            int k = 0;
            if (lane == 0) {
                while (k < pa.n_slots && pa.slot_t[(int64_t)k * n_envs + n] >= 0) ++k;
                if (k == pa.n_slots) {   // contract broken: counted (the agent raises), the last slot is reused
                    atomicAdd(pa.overflow, 1);
                    k = pa.n_slots - 1;
                }
                pa.slot_t[(int64_t)k * n_envs + n] = t;
            }
            k = __shfl(k, 0, 64);
            if (lane < D)
                pa.slot_obs[((int64_t)k * n_envs + n) * D + lane] =
                    obs_norm1(pa.slot_from_next ? eo.sn : eo.sv, m, v, pa.obs_clip);
        }
        if (last && lane < D) pa.boot_norm[n * pa.ld_norm + lane] = obs_norm1(eo.sv, m, v, pa.obs_clip);
        if (rms && lane < D) {
            const double dv = (double)eo.sn - (double)m;
            rp = dv;
            rq = dv * dv;
        }
    }
    if (lane == 0) {
        s_pp[wave][0] = cnt;
        s_pp[wave][1] = sm;
        s_pp[wave][2] = sq;
    }
    if (rms && lane < D) {
        s_pp[wave][3 + lane] = rp;
        s_pp[wave][3 + D + lane] = rq;
    }
    __syncthreads();
    const int tid = threadIdx.x;
    const unsigned nblk = gridDim.x, G = (nblk + kPostGrp - 1) / kPostGrp;
    const int probe = g_k14f_probe;
    if (tid < P)
        xpa_store_agent(pa.part + (int64_t)blockIdx.x * P + tid, ((s_pp[0][tid] + s_pp[1][tid]) + s_pp[2][tid]) + s_pp[3][tid]);
    if (probe & 1) return;
    xpa_drain();
    __syncthreads();
    const unsigned g = blockIdx.x / kPostGrp, g0 = g * kPostGrp;
    const int gn = (int)min((unsigned)kPostGrp, nblk - g0);
    if (tid == 0) s_last = xpa_ticket(pa.tickets + kTicketStride * (1 + g)) == (unsigned)(gn - 1);
    __syncthreads();
    if (!s_last) return;
    if (probe & 2) {
        if (tid == 0) pa.tickets[kTicketStride * (1 + g)] = 0u;
        return;
    }
    // the group's partials: thread (chunk j, column i) sums a contiguous run of blocks in order, then the runs in order
    const int nch = min(4, 256 / P);
    const int i = tid % P, j = tid / P;
    if (j < nch) {
        const int per = (gn + nch - 1) / nch;
        const int lo = j * per, hi = min(gn, lo + per);
        double acc = 0.0;
        for (int b0 = lo; b0 < hi; b0 += 16) {
            double x[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                x[u] = b0 + u < hi ? xpa_load_agent(pa.part + (int64_t)(g0 + b0 + u) * P + i) : 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (b0 + u < hi) acc += x[u];
        }
        s_ch[j][i] = acc;
    }
    __syncthreads();
    if (tid < P) {
        double a = s_ch[0][tid];
        for (int jj = 1; jj < nch; ++jj) a += s_ch[jj][tid];
        xpa_store_agent(pa.part + (int64_t)(nblk + g) * P + tid, a);
    }
    if (tid == 0) pa.tickets[kTicketStride * (1 + g)] = 0u;   // every block of the group has taken its ticket
    if (probe & 4) return;
    xpa_drain();
    __syncthreads();
    if (tid == 0) s_last = xpa_ticket(pa.tickets) == G - 1;
    __syncthreads();
    if (!s_last) return;
    // the last group: the group partials in group order
    if (tid < P) {
        double a = 0.0;
        for (unsigned b0 = 0; b0 < G; b0 += 16) {
            double x[16];
#pragma unroll
            for (unsigned u = 0; u < 16; ++u)
                x[u] = b0 + u < G ? xpa_load_agent(pa.part + (int64_t)(nblk + b0 + u) * P + tid) : 0.0;
#pragma unroll
            for (unsigned u = 0; u < 16; ++u)
                if (b0 + u < G) a += x[u];
        }
        s_ch[0][tid] = a;
    }
    const double c0 = rms ? *pa.obs_count : 0.0;
    __syncthreads();
    if (rms && tid < D) rms_merge_col(s_ch[0][3 + tid], s_ch[0][3 + D + tid], (double)n_envs, c0, pa.obs_mean, pa.obs_var, tid);
    if (tid == 0) {
        if (rms) *pa.obs_count = c0 + (double)n_envs;
        ret_rms_merge(s_ch[0][0], s_ch[0][1], s_ch[0][2], pa.ret_mean, pa.ret_var, pa.ret_count);
        pa.cur->ptr = (int32_t)((t + 1) % T);
        pa.cur->step = pa.cur->step + 1u;
        pa.tickets[0] = 0u;
    }
}

// MODE: 0 Gaussian sample, 1 Categorical sample, 2 value only (v_out[n]).
constexpr int kRolloutKMax = 32;  // head width limit of K14 (lanes < K draw the Gaussian dimensions)
// ENV (Gaussian only): the SynthBox env step of the same env fused after the sample — pre = [W | U] (s | clip(a))
// from the state row and the lanes' clipped actions (fixed k order), then K7's body: no env GEMM and no K7
// launch.  Needs D <= 64 (one state dim per lane).
// r05: with n_envs % 64 == 0, K14E's block b (on XCD b % 8) takes the 8-env granule G = 8 (m >> 1) + (b & 7), m = b >> 3,
// half m & 1: granule G lies on XCD G % 8 — where the rollout trunk's 8-row tile G was written (thin_fwd_norm: block = tile)
// and K40R's XCD-mapped row tiles read and write it — so the z rows and the next step's observation rows stay in one
// XCD's L2 from producer to consumer.  Any env order gives the same per-env results.
__device__ __forceinline__ int64_t xcd_env(int64_t b, int wave, int64_t n_envs) {
    if ((n_envs & 63) != 0) return b * 4 + wave;
    const int64_t m = b >> 3, G = 8 * (m >> 1) + (b & 7);
    return 8 * G + 4 * (m & 1) + wave;
}

// POST (K14F, r06, with MODE 0 + ENV): k14f_tail after the env step; every wave of the block reaches it (waves past
// n_envs skip the env body only)
template <int MODE, int ACT, bool ENV = false, bool POST = false>
__global__ __launch_bounds__(256) void rollout_policy_head_kernel(
    int64_t n_envs, int K, int64_t T, const float *__restrict__ za, const float *__restrict__ zc, int64_t ld,
    float slope, const float *__restrict__ Wa, const float *__restrict__ ba, const float *__restrict__ Wc,
    const float *__restrict__ bc, const float *__restrict__ logstd, const xpa_cursor_t *cur,   // POST: also pa.cur
    uint32_t seed, float act_clip, float *__restrict__ buf_act, float *__restrict__ buf_logp,
    float *__restrict__ buf_val, float *__restrict__ env_in, int64_t ld_env, float *__restrict__ v_out,
    SynthEnvArgs env, PostArgs pa = PostArgs{}) {
    static_assert(!POST || (MODE == 0 && ENV), "K14F is the Gaussian env-fused form");
    __shared__ float s_head[4][kRolloutKMax];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n = ENV ? xcd_env(blockIdx.x, wave, n_envs) : (int64_t)blockIdx.x * 4 + wave;
    const bool valid = n < n_envs;
    if (!POST && !valid) return;  // wave-uniform
    EnvRowOut eo{0.f, 0.f, 0.f, false, false};
    if (valid) {
        // ENV: the env's state row, counters and the first kPreW rows of [W | U]^T are loaded first, so their
        // latency hides under the head arithmetic
        constexpr int kPreW = 24;
        float xs = 0.f, wreg[ENV ? kPreW : 1];
        int e_t = 0;
        uint32_t e_ep = 0u;
        float e_score = 0.f;
        int dl = 0;
        if constexpr (ENV) {
            dl = lane < env.D ? lane : 0;
            xs = lane < env.D ? env.state[n * env.ld_state + lane] : 0.f;
            e_t = env.ep_step[n];
            e_ep = env.ep_index[n];
            e_score = env.ep_score[n];
#pragma unroll
            for (int j = 0; j < kPreW; ++j) {  // unconditional loads (clamped row): no branch + wait per element
                const int jj = j < env.D + K ? j : env.D + K - 1;
                wreg[j] = env.wt[jj * env.D + dl];
            }
        }
        const float4 hc = xpa_act4<ACT>(*reinterpret_cast<const float4 *>(zc + n * ld + 4 * lane), slope);
        const float v = wave_allsum_f(xpa_dot4(hc, *reinterpret_cast<const float4 *>(Wc + 4 * lane))) + bc[0];
        if (MODE == 2) {
            if (lane == 0) v_out[n] = v;
            return;
        }
        const float4 h = xpa_act4<ACT>(*reinterpret_cast<const float4 *>(za + n * ld + 4 * lane), slope);
        float mine = 0.f;  // lane o keeps head[o]
        for (int o = 0; o < K; ++o) {
            const float p = wave_allsum_f(xpa_dot4(h, *reinterpret_cast<const float4 *>(Wa + o * 256 + 4 * lane))) + ba[o];
            if (lane == o) mine = p;
            if (MODE == 1 && lane == 0) s_head[wave][o] = p;
        }
        if (MODE == 1) {
            if (lane == 0) cat_sample_store(n, K, T, s_head[wave], v, cur, seed, buf_act, buf_logp, buf_val, env_in, ld_env);
            return;
        }
        // Gaussian: lane a draws dimension a (the K3 arithmetic); lane 0 adds the log-prob terms in
        // dimension order, so the sum is bitwise K3's sequential one.
        const int64_t cell = n * T + cur->ptr;
        float term_a = 0.f, xclip = 0.f;
        if (lane < K) {
            const int a = lane;
            const uint32_t step = cur->step;
            const uint32_t h1 = xpa_hash4(seed ^ kSaltAct, step, (uint32_t)n, (uint32_t)(2 * a));
            const uint32_t h2 = xpa_hash4(seed ^ kSaltAct, step, (uint32_t)n, (uint32_t)(2 * a + 1));
            const float u1 = 1.0f - xpa_u01(h1);
            const float u2 = xpa_u01(h2);
            const float eps = sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
            const float sc = expf(logstd[a]);
            const float x = mine + sc * eps;
            const float diff = x - mine;
            term_a = -(diff * diff) / (2.0f * sc * sc) - logf(sc) - 0.91893853320467274178f;
            buf_act[cell * K + a] = x;
            xclip = fminf(fmaxf(x, -act_clip), act_clip);
            env_in[n * ld_env + a] = xclip;
        }
        float logp = 0.f;
        for (int a = 0; a < K; ++a) logp += __shfl(term_a, a, 64);
        if (lane == 0) {
            buf_logp[cell] = logp;
            buf_val[cell] = v;
        }
        if constexpr (ENV) {
            // pre = [W | U] (s | clip(a)) for state dim `lane`: one fmaf chain over j < D + K in order
            const int D = env.D, J = D + K;
            float pre = 0.f;
#pragma unroll
            for (int j = 0; j < kPreW; ++j) {
                if (j < J) {  // uniform
                    const float v = __shfl(j < D ? xs : xclip, j < D ? j : j - D, 64);
                    if (lane < D) pre = fmaf(v, wreg[j], pre);
                }
            }
            for (int j = kPreW; j < J; ++j) {
                const float v = __shfl(j < D ? xs : xclip, j < D ? j : j - D, 64);
                const float w = env.wt[j * D + dl];
                if (lane < D) pre = fmaf(v, w, pre);
            }
            eo = synthbox_env_row(n, lane, env, [&](int) { return pre; }, e_t, e_ep, e_score);
        }
    }
    if constexpr (POST) k14f_tail(pa, env.D, eo, valid, n, n_envs, T, lane, wave);
}

// ---------------------------------------------------------------------------------------------
// K7 SynthBox env step (one wave per env, lanes over the state dims)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void synthbox_step_kernel(const float *__restrict__ pre, SynthEnvArgs e,
                                                            int64_t n_envs) {
    const int64_t n = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (n >= n_envs) return;  // wave-uniform
    synthbox_env_row(n, lane, e, [&](int d) { return pre[n * e.D + d]; }, e.ep_step[n], e.ep_index[n], e.ep_score[n]);
}

// ---------------------------------------------------------------------------------------------
// K8 post-step bookkeeping (single block)
// ---------------------------------------------------------------------------------------------
// One env per thread over ceil(n_envs / 256) blocks (the scattered column writes spread over the chip);
// each block writes its finished-return moments (count, sum, sum of squares; f64) to `partials`, and
// the last block to arrive (atomic ticket) merges them in block order into ret_rms, advances the
// cursor and resets the ticket to 0 (graph replays see a fresh ticket).
// DEFER: no v_boot; a mid-buffer truncation of env n copies its normalised final observation row
// (boot_obs) into the env's first free slot k < n_slots (slot_obs[k n_envs + n], slot_t[k n_envs + n] = t);
// with every slot taken it counts in *overflow (the agent sizes n_slots from the env's time limit so that
// this cannot happen: at most ceil((T - 1) / max_episode_steps) mid-buffer truncations per rollout);
// bootstraps are written afterwards by xpa_rollout_bootstrap_fixup.
constexpr int kPostThreads = 256;
// NORM (with DEFER): boot_obs holds the RAW final observations; the kernel normalises them with the obs
// running statistics (obs_normalize_kernel's exact arithmetic) where it keeps a truncation row, and at the
// rollout's last step writes every env's normalised final observation into boot_norm — the second
// normalise launch of each env step is folded in here.

// K8's per-env body (shared with K32): reward normalisation, buffer column t, closures / kept truncation rows,
// the return tracker (R in, the new running return out); (cnt, sum, sumsq) = the env's contribution to ret_rms's
// batch moments.
template <bool DEFER, bool NORM>
__device__ __forceinline__ float post_env(
    int64_t n, int64_t n_envs, int64_t T, int32_t t, bool last, float rstd, float r, bool te, bool tr, float vb,
    float R, float *__restrict__ buf_rew, float *__restrict__ buf_term,
    uint8_t *__restrict__ buf_closed, float *__restrict__ buf_boot, float gamma, int mask_returns, int use_rewnorm,
    float rew_range, int atari_lifeloss, const float *__restrict__ boot_obs, int64_t ld_boot, int64_t dim,
    float *__restrict__ slot_obs, int *__restrict__ slot_t, int n_slots, int *__restrict__ overflow,
    const float *__restrict__ obs_mean, const float *__restrict__ obs_var, float obs_clip,
    float *__restrict__ boot_norm, int64_t ld_norm, double &cnt, double &sum, double &sumsq,
    const float *__restrict__ slot_src = nullptr, int64_t ld_slot = 0) {
    const int64_t cell = n * T + t;
    buf_rew[cell] = use_rewnorm ? fminf(fmaxf(r / rstd, -rew_range), rew_range) : r;
    buf_term[cell] = te ? 1.f : 0.f;
    const bool done = te || tr;
    const bool close = last || (done && !(atari_lifeloss && !tr));
    buf_closed[cell] = close ? 1 : 0;
    buf_boot[cell] = close ? (te ? 0.f : vb) : 0.f;
    if (DEFER && close && !te && !last) {  // mid-buffer truncation: keep the row for later
        int k = 0;
        while (k < n_slots && slot_t[(int64_t)k * n_envs + n] >= 0) ++k;
        if (k == n_slots) {  // contract broken: counted (the agent raises), the last slot is reused
            atomicAdd(overflow, 1);
            k = n_slots - 1;
        }
        const int64_t sl = (int64_t)k * n_envs + n;
        slot_t[sl] = (int)t;
        // the row the bootstrap is formed from: the final observation (PPO), or with slot_src the env's next
        // (reset) observation — A2C's critic call sees obs[i] = reset_obs (a2c_agent.py:88-95)
        const float *src = slot_src ? slot_src + n * ld_slot : boot_obs + n * ld_boot;
        for (int64_t d = 0; d < dim; ++d)
            slot_obs[sl * dim + d] = NORM ? obs_norm1(src[d], obs_mean[d], obs_var[d], obs_clip) : src[d];
    }
    if (NORM && last)
        for (int64_t d = 0; d < dim; ++d)
            boot_norm[n * ld_norm + d] = obs_norm1(boot_obs[n * ld_boot + d], obs_mean[d], obs_var[d], obs_clip);
    float Rk = mask_returns ? (te ? 0.f : gamma * R) + r : gamma * R + r;
    if (done) {
        cnt = 1.0;
        sum = (double)Rk;
        sumsq = (double)Rk * (double)Rk;
        Rk = 0.f;
    }
    return Rk;  // the env's running return
}


// RMS (r05): the NEXT step's obs_rms.update folded in — each block also sums (x - mean) and its square over its envs'
// rows of the observation the env step just produced (f64; the block's 4 waves' sums in order), in
// rms_partials_kernel's partial layout, and the last block runs rms_merge_body after the ret_rms merge.  The next
// step then normalises with the merged statistics and needs no rms launch of its own (the reference updates obs_rms with
// the observation before acting on it: ppoclip_agent.py:62-63, statistic_tools.py:86-112).  obs_dim <= 64.
constexpr int kPostRmsMax = 64;
template <bool DEFER, bool NORM = false, bool RMS = false>
__global__ __launch_bounds__(kPostThreads) void rollout_post_kernel(
    int64_t n_envs, int64_t T, const float *__restrict__ rew, const uint8_t *__restrict__ term,
    const uint8_t *__restrict__ trunc, const float *__restrict__ v_boot, xpa_cursor_t *__restrict__ cur,
    float *__restrict__ ret_mean, float *__restrict__ ret_var, double *__restrict__ ret_count,
    float *__restrict__ returns, float *__restrict__ buf_rew, float *__restrict__ buf_term,
    uint8_t *__restrict__ buf_closed, float *__restrict__ buf_boot, float gamma, int mask_returns, int use_rewnorm,
    float rew_range, int atari_lifeloss, const float *__restrict__ boot_obs, int64_t ld_boot, int64_t dim,
    float *__restrict__ slot_obs, int *__restrict__ slot_t, int n_slots, int *__restrict__ overflow,
    double *__restrict__ partials,
    unsigned int *__restrict__ ticket, const float *__restrict__ obs_mean = nullptr,
    const float *__restrict__ obs_var = nullptr, float obs_clip = 0.f, float *__restrict__ boot_norm = nullptr,
    int64_t ld_norm = 0, const float *__restrict__ slot_src = nullptr, int64_t ld_slot = 0,
    const float *__restrict__ v_boot_mid = nullptr, const float *__restrict__ rms_x = nullptr, int64_t rms_ld = 0,
    int rms_dim = 0, double *__restrict__ rms_part = nullptr, float *rms_mean = nullptr,
    float *__restrict__ rms_var = nullptr, double *__restrict__ rms_count = nullptr) {
    __shared__ double s_red[kPostThreads / 64];
    __shared__ bool s_last;
    const int32_t t = cur->ptr;
    const float rstd = fminf(fmaxf(sqrtf(*ret_var), 0.1f), 100.0f);
    const bool last = (t == (int32_t)(T - 1));
    double cnt = 0.0, sum = 0.0, sumsq = 0.0;
    const int64_t n = (int64_t)blockIdx.x * kPostThreads + threadIdx.x;
    if (n < n_envs)
        returns[n] = post_env<DEFER, NORM>(n, n_envs, T, t, last, rstd, rew[n], term[n] != 0, trunc[n] != 0,
                              DEFER ? 0.f : (v_boot_mid && !last ? v_boot_mid[n] : v_boot[n]), returns[n], buf_rew, buf_term, buf_closed, buf_boot, gamma,
                              mask_returns, use_rewnorm, rew_range, atari_lifeloss, boot_obs, ld_boot, dim, slot_obs,
                              slot_t, n_slots, overflow, obs_mean, obs_var, obs_clip, boot_norm, ld_norm, cnt, sum,
                              sumsq, slot_src, ld_slot);
    constexpr int nw = kPostThreads / 64;
    if constexpr (RMS) {   // this block's partial of the next observation's moments around the running mean
        // 16 columns at a time: the block's rows staged in LDS, then thread (g, j) sums rows g, g + 16, ... of column j
        // in f64 (x - mean exact in f64) and the 16 row groups are added in order
        __shared__ float s_x[kPostThreads][17];
        __shared__ double s_p[16][16], s_q[16][16];
        const int j = threadIdx.x & 15, g = threadIdx.x >> 4;
        for (int c0 = 0; c0 < rms_dim; c0 += 16) {
            const int nc = rms_dim - c0 < 16 ? rms_dim - c0 : 16;
            const int64_t nr = n < n_envs ? n : 0;
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = rms_x[nr * rms_ld + c0 + (u < nc ? u : 0)];
#pragma unroll
            for (int u = 0; u < 16; ++u) s_x[threadIdx.x][u] = v[u];
            __syncthreads();
            double sp = 0.0, sq = 0.0;
            if (j < nc) {
                const double mu = (double)rms_mean[c0 + j];
                for (int r = g; r < kPostThreads; r += 16) {
                    if ((int64_t)blockIdx.x * kPostThreads + r >= n_envs) break;
                    const double d = (double)s_x[r][j] - mu;
                    sp += d;
                    sq += d * d;
                }
            }
            s_p[g][j] = sp;
            s_q[g][j] = sq;
            __syncthreads();
            if ((int)threadIdx.x < nc) {
                double a = s_p[0][threadIdx.x], b = s_q[0][threadIdx.x];
#pragma unroll
                for (int w = 1; w < 16; ++w) {
                    a += s_p[w][threadIdx.x];
                    b += s_q[w][threadIdx.x];
                }
                xpa_store_agent(rms_part + (int64_t)blockIdx.x * rms_dim + c0 + threadIdx.x, a);
                xpa_store_agent(rms_part + ((int64_t)gridDim.x + blockIdx.x) * rms_dim + c0 + threadIdx.x, b);
            }
            __syncthreads();   // s_x / s_p reused by the next 16 columns
        }
    }
    cnt = xpa_block_sum(cnt, s_red, nw);
    sum = xpa_block_sum(sum, s_red, nw);
    sumsq = xpa_block_sum(sumsq, s_red, nw);
    if (RMS) {
        xpa_drain();        // every thread's rms partial stores complete before thread 0's ticket
        __syncthreads();
    }
    if (threadIdx.x == 0) {  // sc1 stores, drained before the ticket (no L2 write-back fence)
        xpa_store_agent(partials + 3 * blockIdx.x, cnt);
        xpa_store_agent(partials + 3 * blockIdx.x + 1, sum);
        xpa_store_agent(partials + 3 * blockIdx.x + 2, sumsq);
        xpa_drain();
        s_last = xpa_ticket(ticket) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    if constexpr (RMS) {   // the next observation's obs_rms merge (all of the last block's threads), then ret_rms
        rms_merge_body(rms_part, gridDim.x, n_envs, rms_dim, rms_mean, rms_var, rms_count);
        __syncthreads();
    }
    // all of the last block's threads load the partials at once (one round trip), thread 0 sums them in
    // block order (deterministic)
    __shared__ double s_pp[3 * 1024];
    const bool staged = gridDim.x <= 1024;
    if (staged)
        for (unsigned i = threadIdx.x; i < 3 * gridDim.x; i += kPostThreads) s_pp[i] = xpa_load_agent(partials + i);
    __syncthreads();
    if (threadIdx.x != 0) return;
    double c = 0.0, s1 = 0.0, s2 = 0.0;
    for (unsigned g = 0; g < gridDim.x; ++g) {  // fixed order -> deterministic
        c += staged ? s_pp[3 * g] : xpa_load_agent(partials + 3 * g);
        s1 += staged ? s_pp[3 * g + 1] : xpa_load_agent(partials + 3 * g + 1);
        s2 += staged ? s_pp[3 * g + 2] : xpa_load_agent(partials + 3 * g + 2);
    }
    ret_rms_merge(c, s1, s2, ret_mean, ret_var, ret_count);
    cur->ptr = (int32_t)((t + 1) % T);
    cur->step = cur->step + 1u;
    *ticket = 0u;
}

// ---------------------------------------------------------------------------------------------
// K32 — `steps` device env steps of a small-MLP Categorical agent on CartPole in one launch (one workgroup):
// obs RMS (K5) -> normalise (obs_normalize) -> MLP forward -> K3 sample/store -> K18 env step -> K8 (deferred,
// NORM).  The RMS sums, the merge, the normalisation, the sampler, the env and the post step are the multi-kernel
// path's own code or arithmetic (one RMS partial block: rows summed per (row group, column) and the groups in
// order, as rms_partials_kernel<., 256> does for n <= 256); the weight rows the forward needs stay in VGPRs for
// the whole launch.  C1: 8 envs, ~10 launches x 128 steps per rollout -> one launch.
// ---------------------------------------------------------------------------------------------
constexpr int kRoThreads = 256;
constexpr int kRoLdsMax = 16384;  // floats of dynamic LDS (64 KiB: no attribute needed)

__host__ __device__ constexpr int ro_r4(int x) { return (x + 3) & ~3; }

struct RoLayout {
    int sy, sz, sbo, total;
};
// sy: the normalised observations [N][4]; sz: the output layers' partial sums [wave][N][K + 1]; sbo: biases
__host__ __device__ inline RoLayout ro_layout(int N, int D, int H0, int H1, int H2, int K) {
    RoLayout l;
    const int K1 = K + 1;
    (void)H0;
    (void)H1;
    (void)H2;
    l.sy = 0;
    l.sz = ro_r4(N * D);
    l.sbo = ro_r4(l.sz + 4 * N * K1);
    l.total = ro_r4(l.sbo + K1);
    return l;
}

// Sum over the wave's 64 lanes on DPP lane moves (no LDS round trip); the total lands in lane 63.  Lanes a move
// leaves out (row_mask) add 0.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float ro_dpp(float src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, src), CTRL, ROW_MASK, 0xf,
                                                                 false));
}
__device__ __forceinline__ float ro_wave_sum63(float v) {
    v += ro_dpp<0xB1>(v);        // quad_perm [1, 0, 3, 2]
    v += ro_dpp<0x4E>(v);        // quad_perm [2, 3, 0, 1]
    v += ro_dpp<0x141>(v);       // row_half_mirror: sums of 8
    v += ro_dpp<0x140>(v);       // row_mirror: sums of 16
    v += ro_dpp<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v += ro_dpp<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return v;
}

// Sum over the 16 lanes of each DPP row (every lane gets its row's sum).
__device__ __forceinline__ float ro_row_sum16(float v) {
    v += ro_dpp<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += ro_dpp<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += ro_dpp<0x141>(v);  // row_half_mirror: sums of 8
    v += ro_dpp<0x140>(v);  // row_mirror: sums of 16
    return v;
}
typedef float ro_f32x4 __attribute__((ext_vector_type(4)));

// K8's f64 wave butterfly (xpa_wave_sum) when only lanes [0, n) hold values (the rest +0): the steps whose partner
// lanes are all empty add +0 and are skipped.
__device__ __forceinline__ double ro_wave_sum_first(double v, int n) {
    for (int o = 32; o > 0; o >>= 1)
        if (o < n) v += __shfl_xor(v, o, 64);
    return v;
}

template <int ACT>
__device__ __forceinline__ float ro_act(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

template <int ACT, int H0>
__global__ __launch_bounds__(kRoThreads) void small_rollout_cartpole_kernel(XpaSmallRolloutArgs a) {
    extern __shared__ float lds[];
    __shared__ double s_sum[kRoThreads], s_sq[kRoThreads];
    __shared__ double s_red[kRoThreads / 64];
    __shared__ float s_mean[4], s_var[4];
    __shared__ float s_obs[256 * 4];  // the raw observations of the step
    __shared__ float s_rstd;
    constexpr int D = 4;  // CartPole
    const int tid = threadIdx.x;
    const int N = a.n_envs, H1 = a.h1, H2 = a.h2, K = a.k, K1 = a.k + 1, U = a.h1 + a.h2;
    const int T = a.horizon;
    const RoLayout L = ro_layout(N, D, H0, H1, H2, K);
    float *sy = lds + L.sy, *sz = lds + L.sz, *sbo = lds + L.sbo;
    const XpaCartPoleEnv env{a.env_state,   a.env_obs,   a.ld_obs,     a.final_obs,  a.env_rew,
                             a.env_term,    a.env_trunc, a.ep_step,    a.ep_index,   a.ep_score,
                             a.ep_last_score, a.ep_last_len, a.env_seed, a.max_episode_steps,
                             cartpole::kThetaThreshold};
    if (tid < K1) sbo[tid] = tid < K ? a.ba[tid] : a.bc[0];
    // The forward on v_mfma_f32_16x16x4_f32: [16-row tile of envs] x [actor | critic hidden units], K = h0.  Wave w
    // owns the unit tiles w and w + 4 (16 units each) with their weight rows in VGPRs (B operand, loaded once per
    // launch); lane (q, i) forms the A operand itself — h0[row i][4 kk + q] of the representation layer, from the
    // normalised row in LDS — so h0 never goes through LDS; the output layers are per-lane partial dot products over
    // the lane's units, summed over the 16 lanes of a DPP row and then over the waves (LDS, fixed order).
    const int wave = tid >> 6, lane = tid & 63;
    const int li = lane & 15, lq = lane >> 4;
    constexpr int KK = H0 / 4;
    const int UT = U >> 4;   // unit tiles (4, 6 or 8)
    float4 w0k[KK];
    float b0k[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        const int k = 4 * kk + lq;
        w0k[kk] = make_float4(a.W0[k * D], a.W0[k * D + 1], a.W0[k * D + 2], a.W0[k * D + 3]);
        b0k[kk] = a.b0[k];
    }
    float bw[2][KK], b12[2], wo[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int tile = wave + 4 * j;
        const bool tok = tile < UT;
        const int u = tok ? 16 * tile + li : 0;
        const bool actor = u < H1;
        const float *wr = actor ? a.W1 + u * H0 : a.W2 + (u - H1) * H0;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) bw[j][kk] = tok ? wr[4 * kk + lq] : 0.f;
        b12[j] = tok ? (actor ? a.b1[u] : a.b2[u - H1]) : 0.f;
#pragma unroll
        for (int o = 0; o < 3; ++o)
            wo[j][o] = !tok || o >= K1 ? 0.f : (o < K ? (actor ? a.Wa[o * H1 + u] : 0.f) : (actor ? 0.f : a.Wc[u - H1]));
    }

    // state that lives across the steps of the launch: each env's CartPole state and running return (thread n),
    // the raw observations and obs statistics (LDS), the obs count (every thread), the return statistics (thread 0)
    cartpole::Local es{};
    float R = 0.f;
    if (tid < N) {
        es = cartpole::load(env, tid);
        R = a.returns[tid];
#pragma unroll
        for (int d = 0; d < 4; ++d) s_obs[tid * 4 + d] = a.env_obs[tid * a.ld_obs + d];
    }
    if (tid < D) {
        s_mean[tid] = a.obs_mean[tid];
        s_var[tid] = a.obs_var[tid];
    }
    double ocount = *a.obs_count;
    float rmean = 0.f, rvar = 0.f;
    double rcount = 0.0;
    if (tid == 0) {
        rmean = *a.ret_mean;
        rvar = *a.ret_var;
        rcount = *a.ret_count;
        s_rstd = fminf(fmaxf(sqrtf(rvar), 0.1f), 100.0f);
    }
    int32_t t = a.cursor->ptr;
    uint32_t step = a.cursor->step;
    int64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0, st_t0 = 0;
#define XPA_RO_STAMP(i_)                                                    \
    do {                                                                    \
        if (a.stamps && tid == 0) {                                         \
            const int64_t now_ = (int64_t)__builtin_amdgcn_s_memtime();     \
            st_acc[i_] += now_ - st_prev;                                   \
            st_prev = now_;                                                 \
        }                                                                   \
    } while (0)
    __syncthreads();
    if (a.stamps && tid == 0) st_prev = st_t0 = (int64_t)__builtin_amdgcn_s_memtime();
    constexpr int kGroups = kRoThreads / D;  // rms_partials_kernel<., 256>'s row groups at dim 4
    for (int s = 0; s < a.steps; ++s) {
        const bool last = t == T - 1;
        // (a) obs_rms.update(obs): xpa_rms_update with one partial block
        if (a.use_obsnorm) {
            double ts = 0.0, tq = 0.0;
            if (N <= kGroups) {
                // one row per row group: the group-ordered sums are the row sums in row order (every group sum is
                // 0 + v or 0 + v * v, rounded once; the empty groups add +0)
                if (tid < D) {
#pragma clang fp contract(off)
                    const float sh = s_mean[tid];
                    for (int r = 0; r < N; ++r) {
                        const double v = (double)s_obs[r * 4 + tid] - (double)sh;
                        const double vv = v * v;
                        ts = ts + v;
                        tq = tq + vv;
                    }
                }
            } else {
                const int c = tid % D, gsub = tid / D;
                double sm = 0.0, q = 0.0;
                const float sh = s_mean[c];
                for (int r = gsub; r < N; r += kGroups) {
                    const double v = (double)s_obs[r * 4 + c] - (double)sh;
                    sm += v;
                    q += v * v;
                }
                s_sum[tid] = sm;
                s_sq[tid] = q;
                __syncthreads();
                if (tid < D)
                    for (int k = 0; k < kGroups; ++k) {
                        ts += s_sum[k * D + tid];
                        tq += s_sq[k * D + tid];
                    }
            }
            if (tid < D) {
                double s1 = 0.0, q1 = 0.0;  // rms_merge_body over the one partial
                s1 += ts;
                q1 += tq;
                const double n = (double)N, c0 = ocount;
                const double ms = s1 / n;
                const double m0 = (double)s_mean[tid], v0 = (double)s_var[tid];
                const double bm = m0 + ms;
                const double bvar = fmax(q1 / n - ms * ms, 0.0);
                const double tot = c0 + n;
                const double delta = bm - m0;
                const double new_mean = m0 + delta * n / tot;
                const double m2 = v0 * c0 + bvar * n + delta * delta * c0 * n / tot;
                const float fm = (float)new_mean, fv = (float)(m2 / tot);
                a.obs_mean[tid] = fm;
                a.obs_var[tid] = fv;
                s_mean[tid] = fm;
                s_var[tid] = fv;
            }
            ocount = ocount + (double)N;
            if (tid == 0) *a.obs_count = ocount;
            __syncthreads();
        }
        XPA_RO_STAMP(0);
        // (b) normalise into the policy input and buffer column t (obs_normalize_kernel's arithmetic)
        for (int e = tid; e < N * D; e += kRoThreads) {
            const int r = e >> 2, d = e & 3;
            const float y = obs_norm1(s_obs[e], s_mean[d], s_var[d], a.obs_clip);
            sy[e] = y;
            a.obs_norm[r * a.ld_norm + d] = y;
            a.buf_obs[((int64_t)r * T + t) * D + d] = y;
        }
        __syncthreads();
        XPA_RO_STAMP(1);
        // (c)-(e) the forward, one 16-row tile of envs at a time
        for (int r0 = 0; r0 < N; r0 += 16) {
            const int ra = r0 + li < N ? r0 + li : N - 1;   // this lane's A row (rows past N: results unused)
            const float4 y = *reinterpret_cast<const float4 *>(sy + ra * D);
            float av[KK];
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                float z = b0k[kk];
                z = fmaf(w0k[kk].x, y.x, z);
                z = fmaf(w0k[kk].y, y.y, z);
                z = fmaf(w0k[kk].z, y.z, z);
                z = fmaf(w0k[kk].w, y.w, z);
                av[kk] = ro_act<ACT>(z, a.slope);
            }
            ro_f32x4 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[j] = ro_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bw[j][kk], acc[j], 0, 0, 0);
            // D element r of lane (q, i): row r0 + 4 q + r, unit 16 tile + i
            float part[4][3];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int o = 0; o < 3; ++o) {
                    float pv = 0.f;
#pragma unroll
                    for (int j = 0; j < 2; ++j) pv = fmaf(wo[j][o], ro_act<ACT>(acc[j][r] + b12[j], a.slope), pv);
                    part[r][o] = ro_row_sum16(pv);
                }
            if (li == 0)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = r0 + 4 * lq + r;
                    if (m < N)
                        for (int o = 0; o < K1; ++o) sz[(wave * N + m) * K1 + o] = part[r][o];
                }
        }
        __syncthreads();
        XPA_RO_STAMP(4);
        // (f) sample + store, env step, post step (one thread per env)
        double cnt = 0.0, sum = 0.0, sumsq = 0.0;
        if (tid < N) {
            float z[3];
            for (int o = 0; o < K1; ++o) {
                float v = sbo[o];
                for (int w = 0; w < 4; ++w) v += sz[(w * N + tid) * K1 + o];
                z[o] = v;
            }
            const int pick = cat_sample_store_at(tid, K, T, t, step, z, z[K], a.seed, a.buf_act, a.buf_logp,
                                                 a.buf_val, a.act_in, a.ld_act);
            bool te, tr;
            float o[4];
            const float r = cartpole::step(env, tid, pick, es, &te, &tr, o);
#pragma unroll
            for (int d = 0; d < 4; ++d) s_obs[tid * 4 + d] = o[d];
            R = post_env<true, true>(tid, N, T, t, last, s_rstd, r, te, tr, 0.f, R, a.buf_rew, a.buf_term,
                                     a.buf_closed, a.buf_boot, a.gamma, a.mask_returns, a.use_rewnorm, a.rew_range,
                                     0, a.final_obs, 4, D, a.slot_obs, a.slot_t, a.n_slots, a.overflow, s_mean, s_var,
                                     a.obs_clip, a.boot_norm, a.ld_boot, cnt, sum, sumsq,
                                     a.slot_reset_obs ? a.env_obs : nullptr, a.ld_obs);
            a.returns[tid] = R;
        }
        XPA_RO_STAMP(5);
        // (g) ret_rms over the closed paths: K8's block sums (all envs in wave 0 when N <= 64: the other waves'
        // sums are +0), then its merge
        if (N <= 64) {
            if (tid < 64) {
                const int np2 = N <= 1 ? 1 : 1 << (32 - __builtin_clz(N - 1));  // lanes [0, np2) may hold values
                cnt = 0.0 + ro_wave_sum_first(cnt, np2);
                sum = 0.0 + ro_wave_sum_first(sum, np2);
                sumsq = 0.0 + ro_wave_sum_first(sumsq, np2);
            }
        } else {
            cnt = xpa_block_sum(cnt, s_red, kRoThreads / 64);
            sum = xpa_block_sum(sum, s_red, kRoThreads / 64);
            sumsq = xpa_block_sum(sumsq, s_red, kRoThreads / 64);
        }
        if (tid == 0 && cnt > 0.0) {
            ret_rms_merge_local(cnt, sum, sumsq, rmean, rvar, rcount);
            *a.ret_mean = rmean;
            *a.ret_var = rvar;
            *a.ret_count = rcount;
            s_rstd = fminf(fmaxf(sqrtf(rvar), 0.1f), 100.0f);
        }
        XPA_RO_STAMP(6);
        t = (t + 1) % T;
        step += 1u;
        __syncthreads();  // next observations, statistics and rstd visible to the next step
        XPA_RO_STAMP(7);
    }
#undef XPA_RO_STAMP
    if (a.stamps && tid == 0) {
        for (int i = 0; i < 8; ++i) a.stamps[i] = st_acc[i];
        a.stamps[8] = (int64_t)__builtin_amdgcn_s_memtime() - st_t0;
    }
    if (tid < N) cartpole::store(env, tid, es);
    if (tid == 0) {
        a.cursor->ptr = t;
        a.cursor->step = step;
    }
}

}  // namespace

// ---- K4 --------------------------------------------------------------------------------------------
XPA_API int64_t xpa_gather_num_partials(int64_t batch) { return (batch + kGatherRows - 1) / kGatherRows; }

XPA_API int xpa_gather_minibatch(const int64_t *idx, int64_t batch, int64_t n_rows, const void *obs,
                                 int64_t obs_row_bytes, void *obs_out, const float *adv, double *adv_partials,
                                 int32_t *err, xpa_stream_t stream) {
    if (batch <= 0 || n_rows <= 0 || obs_row_bytes < 0 || !idx) return (int)hipErrorInvalidValue;
    if (obs_row_bytes > 0 && (!obs || !obs_out)) return (int)hipErrorInvalidValue;
    if (adv_partials && !adv) return (int)hipErrorInvalidValue;
    const int64_t blocks = xpa_gather_num_partials(batch);
    hipStream_t s = (hipStream_t)stream;
    const uintptr_t al = (uintptr_t)obs | (uintptr_t)obs_out;
    if (obs_row_bytes >= 4096 && obs_row_bytes % 16 == 0 && al % 16 == 0) {
        const int64_t rv = obs_row_bytes / 16, chunks = (rv + 256 * kWideU - 1) / (256 * kWideU);
        if (batch * chunks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(gather_wide_kernel, dim3((unsigned)(batch * chunks)), dim3(256), 0, s, idx, n_rows,
                           (const u4v *)obs, rv, chunks, (u4v *)obs_out, err);
        if (adv_partials)  // the moments alone (no row copy)
            hipLaunchKernelGGL(gather_rows_kernel<uint4>, dim3((unsigned)blocks), dim3(256), 0, s, idx, batch, n_rows,
                               (const uint4 *)obs, (int64_t)0, (uint4 *)obs_out, adv, adv_partials,
                               (int *)nullptr);
    } else if (obs_row_bytes % 16 == 0 && al % 16 == 0)
        hipLaunchKernelGGL(gather_rows_kernel<uint4>, dim3((unsigned)blocks), dim3(256), 0, s, idx, batch,
                           n_rows, (const uint4 *)obs, obs_row_bytes / 16, (uint4 *)obs_out, adv, adv_partials, err);
    else if (obs_row_bytes % 4 == 0 && al % 4 == 0)
        hipLaunchKernelGGL(gather_rows_kernel<uint32_t>, dim3((unsigned)blocks), dim3(256), 0, s, idx, batch,
                           n_rows, (const uint32_t *)obs, obs_row_bytes / 4, (uint32_t *)obs_out, adv, adv_partials,
                           err);
    else
        hipLaunchKernelGGL(gather_rows_kernel<uint8_t>, dim3((unsigned)blocks), dim3(256), 0, s, idx, batch,
                           n_rows, (const uint8_t *)obs, obs_row_bytes, (uint8_t *)obs_out, adv, adv_partials, err);
    return xpa_launch_status();
}

// r05: K4 into rows of pitch out_row_bytes >= obs_row_bytes (the bytes past each row's obs_row_bytes untouched: the
// C4 trunk's zero-padded K40F operand, 376 -> 384 floats); 16-B vectors only
XPA_API int xpa_gather_minibatch_pitched(const int64_t *idx, int64_t batch, int64_t n_rows, const void *obs,
                                         int64_t obs_row_bytes, void *obs_out, int64_t out_row_bytes,
                                         const float *adv, double *adv_partials, int32_t *err, xpa_stream_t stream) {
    if (batch <= 0 || n_rows <= 0 || obs_row_bytes <= 0 || !idx || !obs || !obs_out || out_row_bytes < obs_row_bytes ||
        obs_row_bytes % 16 || out_row_bytes % 16 || (((uintptr_t)obs | (uintptr_t)obs_out) % 16) ||
        (adv_partials && !adv))
        return (int)hipErrorInvalidValue;
    const int64_t blocks = xpa_gather_num_partials(batch);
    if ((int64_t)kGatherRows * (obs_row_bytes / 16) > 0xffffffffLL) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_rows_kernel<uint4>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, idx, batch,
                       n_rows, (const uint4 *)obs, obs_row_bytes / 16, (uint4 *)obs_out, adv, adv_partials, err,
                       out_row_bytes / 16);
    return xpa_launch_status();
}

// ---- K5 --------------------------------------------------------------------------------------------
XPA_API int64_t xpa_rms_num_partials(int64_t n) { return (n + kRmsRows - 1) / kRmsRows; }

XPA_API int xpa_rms_partials(const float *x, int64_t n, int64_t dim, int64_t ld, const float *shift,
                             double *partials, xpa_stream_t stream) {
    if (n <= 0 || dim <= 0 || ld < dim || !x || !partials) return (int)hipErrorInvalidValue;
    const int64_t np = xpa_rms_num_partials(n);
    if (dim > kRmsWideDim)
        hipLaunchKernelGGL((rms_partials_cols_kernel<false>), dim3((unsigned)np, (unsigned)((dim + 63) / 64)), dim3(1024),
                           0, (hipStream_t)stream, x, n, dim, ld, shift, partials, (float *)nullptr, (float *)nullptr,
                           (double *)nullptr, (unsigned int *)nullptr);
    else
        hipLaunchKernelGGL((rms_partials_kernel<false, 256>), dim3((unsigned)np), dim3(256), 0, (hipStream_t)stream, x,
                           n, dim, ld, shift, partials, (float *)nullptr, (float *)nullptr, (double *)nullptr,
                           (unsigned int *)nullptr);
    return xpa_launch_status();
}

XPA_API int xpa_rms_update(const float *x, int64_t n, int64_t dim, int64_t ld, float *mean, float *var,
                           double *count, double *partials, int32_t *ticket, xpa_stream_t stream) {
    if (n <= 0 || dim <= 0 || ld < dim || !x || !mean || !var || !count || !partials || !ticket)
        return (int)hipErrorInvalidValue;
    const int64_t np = xpa_rms_num_partials(n);
    if (dim > kRmsWideDim)
        hipLaunchKernelGGL((rms_partials_cols_kernel<true>), dim3((unsigned)np, (unsigned)((dim + 63) / 64)), dim3(1024),
                           0, (hipStream_t)stream, x, n, dim, ld, (const float *)mean, partials, mean, var, count,
                           (unsigned int *)ticket);
    else
        hipLaunchKernelGGL((rms_partials_kernel<true, 256>), dim3((unsigned)np), dim3(256), 0, (hipStream_t)stream, x,
                           n, dim, ld, (const float *)mean, partials, mean, var, count, (unsigned int *)ticket);
    return xpa_launch_status();
}

XPA_API int xpa_rms_merge(const double *partials, int64_t n_partials, int64_t n, int64_t dim, float *mean,
                          float *var, double *count, xpa_stream_t stream) {
    if (n <= 0 || dim <= 0 || n_partials <= 0 || !partials || !mean || !var || !count)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(rms_merge_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, n_partials, n, dim,
                       mean, var, count);
    return xpa_launch_status();
}

XPA_API int xpa_obs_normalize(const float *x, int64_t n, int64_t dim, int64_t ldx, const float *mean,
                              const float *var, float clip_range, float *out, int64_t ldo, float *col_out,
                              int64_t col_ld, const xpa_cursor_t *cursor, xpa_stream_t stream) {
    if (n <= 0 || dim <= 0 || ldx < dim || ldo < dim || !x || !mean || !var || !out) return (int)hipErrorInvalidValue;
    if (col_out && (!cursor || col_ld < dim)) return (int)hipErrorInvalidValue;
    const int64_t total = n * dim;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(obs_normalize_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, n, dim, ldx,
                       mean, var, clip_range, out, ldo, col_out, col_ld, cursor);
    return xpa_launch_status();
}

// ---- K3 --------------------------------------------------------------------------------------------
XPA_API int xpa_rollout_sample(int dist, int64_t n_envs, int64_t act_dim, int64_t horizon, const float *head,
                               const float *logstd, const float *v, const xpa_cursor_t *cursor, uint32_t seed,
                               float act_clip, float *buf_act, float *buf_logp, float *buf_val, float *env_in,
                               int64_t ld_env, xpa_stream_t stream) {
    if (n_envs <= 0 || act_dim <= 0 || horizon <= 0 || !head || !v || !cursor || !buf_act || !buf_logp ||
        !buf_val || !env_in || ld_env < act_dim)
        return (int)hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((n_envs + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    if (dist == XPA_DIST_GAUSSIAN) {
        if (!logstd) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(rollout_sample_gauss_kernel, dim3(blocks), dim3(256), 0, s, n_envs, (int)act_dim, horizon,
                           head, logstd, v, cursor, seed, act_clip, buf_act, buf_logp, buf_val, env_in, ld_env);
    } else if (dist == XPA_DIST_CATEGORICAL) {
        if (act_dim < 2) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(rollout_sample_cat_kernel, dim3(blocks), dim3(256), 0, s, n_envs, (int)act_dim, horizon,
                           head, v, cursor, seed, buf_act, buf_logp, buf_val, env_in, ld_env);
    } else {
        return (int)hipErrorInvalidValue;
    }
    return xpa_launch_status();
}

// ---- K7 --------------------------------------------------------------------------------------------
XPA_API int xpa_synthbox_step(int64_t n_envs, int64_t obs_dim, const float *pre, uint32_t seed,
                              int32_t max_episode_steps, float noise, float term_thresh, float reset_scale,
                              float *state, int64_t ld_state, float *final_obs, float *rew, uint8_t *term,
                              uint8_t *trunc, int32_t *ep_step, uint32_t *ep_index, float *ep_score,
                              float *ep_last_score, int32_t *ep_last_len, xpa_stream_t stream) {
    if (n_envs <= 0 || obs_dim <= 0 || ld_state < obs_dim || !pre || !state || !final_obs || !rew || !term ||
        !trunc || !ep_step || !ep_index || !ep_score || !ep_last_score || !ep_last_len)
        return (int)hipErrorInvalidValue;
    SynthEnvArgs e{(int)obs_dim, seed, max_episode_steps, noise, term_thresh, reset_scale, state, ld_state, final_obs,
                   rew, term, trunc, ep_step, ep_index, ep_score, ep_last_score, ep_last_len, nullptr};
    const unsigned blocks = (unsigned)((n_envs + 3) / 4);
    hipLaunchKernelGGL(synthbox_step_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, pre, e, n_envs);
    return xpa_launch_status();
}

// ---- K8 --------------------------------------------------------------------------------------------
XPA_API int64_t xpa_rollout_post_num_blocks(int64_t n_envs) {
    return (n_envs + kPostThreads - 1) / kPostThreads;
}

XPA_API int xpa_rollout_post(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                             const uint8_t *trunc, const float *v_boot, const float *v_boot_mid,
                             xpa_cursor_t *cursor, float *ret_mean,
                             float *ret_var, double *ret_count, float *returns, float *buf_rew, float *buf_term,
                             uint8_t *buf_closed, float *buf_boot, float gamma, int mask_returns, int use_rewnorm,
                             float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
                             xpa_stream_t stream) {
    if (n_envs <= 0 || horizon <= 0 || !rew || !term || !trunc || !v_boot || !cursor || !ret_mean || !ret_var ||
        !ret_count || !returns || !buf_rew || !buf_term || !buf_closed || !buf_boot || !partials || !ticket ||
        xpa_rollout_post_num_blocks(n_envs) > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(rollout_post_kernel<false>, dim3((unsigned)xpa_rollout_post_num_blocks(n_envs)),
                       dim3(kPostThreads), 0, (hipStream_t)stream, n_envs, horizon, rew, term, trunc, v_boot, cursor,
                       ret_mean, ret_var, ret_count, returns, buf_rew, buf_term, buf_closed, buf_boot, gamma,
                       mask_returns, use_rewnorm, rew_range, atari_lifeloss, (const float *)nullptr, (int64_t)0,
                       (int64_t)0, (float *)nullptr, (int *)nullptr, 0, (int *)nullptr, partials, (unsigned *)ticket,
                       (const float *)nullptr, (const float *)nullptr, 0.f, (float *)nullptr, (int64_t)0,
                       (const float *)nullptr, (int64_t)0, v_boot_mid);
    return xpa_launch_status();
}

XPA_API int xpa_rollout_post_deferred(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                                      const uint8_t *trunc, const float *boot_obs, int64_t ld_boot, int64_t obs_dim,
                                      float *slot_obs, int32_t *slot_t, int64_t n_slots, int32_t *overflow,
                                      xpa_cursor_t *cursor, float *ret_mean, float *ret_var, double *ret_count,
                                      float *returns, float *buf_rew, float *buf_term, uint8_t *buf_closed,
                                      float *buf_boot, float gamma, int mask_returns, int use_rewnorm,
                                      float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
                                      xpa_stream_t stream) {
    if (n_envs <= 0 || horizon <= 0 || obs_dim <= 0 || ld_boot < obs_dim || n_slots < 1 || n_slots > horizon ||
        !rew || !term || !trunc || !boot_obs ||
        !slot_obs || !slot_t || !overflow || !cursor || !ret_mean || !ret_var || !ret_count || !returns || !buf_rew ||
        !buf_term || !buf_closed || !buf_boot || !partials || !ticket || xpa_rollout_post_num_blocks(n_envs) > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(rollout_post_kernel<true>, dim3((unsigned)xpa_rollout_post_num_blocks(n_envs)),
                       dim3(kPostThreads), 0, (hipStream_t)stream, n_envs, horizon, rew, term, trunc,
                       (const float *)nullptr, cursor, ret_mean, ret_var, ret_count, returns, buf_rew, buf_term,
                       buf_closed, buf_boot, gamma, mask_returns, use_rewnorm, rew_range, atari_lifeloss, boot_obs,
                       ld_boot, obs_dim, slot_obs, slot_t, (int)n_slots, overflow, partials, (unsigned *)ticket,
                       (const float *)nullptr, (const float *)nullptr, 0.f, (float *)nullptr, (int64_t)0);
    return xpa_launch_status();
}

XPA_API int xpa_rollout_post_deferred_norm(int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term,
                                           const uint8_t *trunc, const float *final_obs, int64_t ld_final,
                                           const float *slot_src, int64_t ld_slot, int64_t obs_dim, const float *obs_mean, const float *obs_var,
                                           float obs_clip, float *boot_norm, int64_t ld_norm, float *slot_obs,
                                           int32_t *slot_t, int64_t n_slots, int32_t *overflow,
                                           xpa_cursor_t *cursor, float *ret_mean,
                                           float *ret_var, double *ret_count, float *returns, float *buf_rew,
                                           float *buf_term, uint8_t *buf_closed, float *buf_boot, float gamma,
                                           int mask_returns, int use_rewnorm, float rew_range, int atari_lifeloss,
                                           double *partials, uint32_t *ticket, xpa_stream_t stream) {
    if (n_envs <= 0 || horizon <= 0 || obs_dim <= 0 || ld_final < obs_dim || ld_norm < obs_dim || n_slots < 1 ||
        n_slots > horizon || (slot_src && ld_slot < obs_dim) || !rew || !term ||
        !trunc || !final_obs || !obs_mean || !obs_var || !boot_norm || !slot_obs || !slot_t || !overflow || !cursor ||
        !ret_mean || !ret_var || !ret_count || !returns || !buf_rew || !buf_term || !buf_closed || !buf_boot ||
        !partials || !ticket || xpa_rollout_post_num_blocks(n_envs) > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((rollout_post_kernel<true, true>), dim3((unsigned)xpa_rollout_post_num_blocks(n_envs)),
                       dim3(kPostThreads), 0, (hipStream_t)stream, n_envs, horizon, rew, term, trunc,
                       (const float *)nullptr, cursor, ret_mean, ret_var, ret_count, returns, buf_rew, buf_term,
                       buf_closed, buf_boot, gamma, mask_returns, use_rewnorm, rew_range, atari_lifeloss, final_obs,
                       ld_final, obs_dim, slot_obs, slot_t, (int)n_slots, overflow, partials, (unsigned *)ticket,
                       obs_mean, obs_var, obs_clip, boot_norm, ld_norm, slot_src, ld_slot);
    return xpa_launch_status();
}

// r05: xpa_rollout_post_deferred_norm with the NEXT step's obs_rms.update folded in (rms_x [n_envs, rms_dim], row
// stride rms_ld: the observation the env step just produced; rms_part f64 [2 * xpa_rollout_post_num_blocks(n_envs),
// rms_dim]; obs_mean / obs_var / obs_count updated in place by the last block, after every block normalised with the
// old statistics).  obs_dim <= 64.
XPA_API int xpa_rollout_post_deferred_norm_rms(
    int64_t n_envs, int64_t horizon, const float *rew, const uint8_t *term, const uint8_t *trunc, const float *final_obs,
    int64_t ld_final, const float *slot_src, int64_t ld_slot, int64_t obs_dim, float *obs_mean, float *obs_var,
    double *obs_count, float obs_clip, float *boot_norm, int64_t ld_norm, float *slot_obs, int32_t *slot_t,
    int64_t n_slots, int32_t *overflow, xpa_cursor_t *cursor, float *ret_mean, float *ret_var, double *ret_count,
    float *returns, float *buf_rew, float *buf_term, uint8_t *buf_closed, float *buf_boot, float gamma,
    int mask_returns, int use_rewnorm, float rew_range, int atari_lifeloss, double *partials, uint32_t *ticket,
    const float *rms_x, int64_t rms_ld, double *rms_part, xpa_stream_t stream) {
    if (n_envs <= 0 || horizon <= 0 || obs_dim <= 0 || obs_dim > kPostRmsMax || ld_final < obs_dim ||
        ld_norm < obs_dim || n_slots < 1 || n_slots > horizon || (slot_src && ld_slot < obs_dim) || !rew || !term ||
        !trunc || !final_obs || !obs_mean || !obs_var || !obs_count || !boot_norm || !slot_obs || !slot_t ||
        !overflow || !cursor || !ret_mean || !ret_var || !ret_count || !returns || !buf_rew || !buf_term ||
        !buf_closed || !buf_boot || !partials || !ticket || !rms_x || rms_ld < obs_dim || !rms_part ||
        xpa_rollout_post_num_blocks(n_envs) > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((rollout_post_kernel<true, true, true>), dim3((unsigned)xpa_rollout_post_num_blocks(n_envs)),
                       dim3(kPostThreads), 0, (hipStream_t)stream, n_envs, horizon, rew, term, trunc,
                       (const float *)nullptr, cursor, ret_mean, ret_var, ret_count, returns, buf_rew, buf_term,
                       buf_closed, buf_boot, gamma, mask_returns, use_rewnorm, rew_range, atari_lifeloss, final_obs,
                       ld_final, obs_dim, slot_obs, slot_t, (int)n_slots, overflow, partials, (unsigned *)ticket,
                       obs_mean, obs_var, obs_clip, boot_norm, ld_norm, slot_src, ld_slot, (const float *)nullptr,
                       rms_x, rms_ld, (int)obs_dim, rms_part, obs_mean, obs_var, obs_count);
    return xpa_launch_status();
}

namespace {
// v = V([slot rows (n_slots x n_envs); last-step rows (n_envs)]): every used slot's bootstrap, then the last column's.
__global__ __launch_bounds__(256) void bootstrap_fixup_kernel(int64_t n_envs, int64_t T, int n_slots,
                                                              const float *__restrict__ v, int *__restrict__ slot_t,
                                                              const float *__restrict__ buf_term,
                                                              float *__restrict__ buf_boot) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= n_envs) return;
    for (int k = 0; k < n_slots; ++k) {
        const int64_t sl = (int64_t)k * n_envs + n;
        const int t = slot_t[sl];
        if (t >= 0 && t < T) buf_boot[n * T + t] = v[sl];
        slot_t[sl] = -1;
    }
    const int64_t last = n * T + T - 1;
    buf_boot[last] = buf_term[last] != 0.f ? 0.f : v[(int64_t)n_slots * n_envs + n];
}
}  // namespace

XPA_API int xpa_rollout_bootstrap_fixup(int64_t n_envs, int64_t horizon, const float *values, int32_t *slot_t,
                                        int64_t n_slots, const float *buf_term, float *buf_boot, xpa_stream_t stream) {
    if (n_envs <= 0 || horizon <= 0 || n_slots < 1 || n_slots > horizon || !values || !slot_t || !buf_term ||
        !buf_boot)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bootstrap_fixup_kernel, dim3((unsigned)((n_envs + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, n_envs, horizon, (int)n_slots, values, slot_t, buf_term, buf_boot);
    return xpa_launch_status();
}

// ---- K14 -------------------------------------------------------------------------------------------
XPA_API int xpa_rollout_policy_head(int dist, int act, int64_t n_envs, int64_t act_dim, int64_t horizon,
                                    int64_t hidden, int64_t ld, const float *z_actor, const float *z_critic,
                                    float slope, const float *w_actor, const float *b_actor, const float *w_critic,
                                    const float *b_critic, const float *logstd, const xpa_cursor_t *cursor,
                                    uint32_t seed, float act_clip, float *buf_act, float *buf_logp, float *buf_val,
                                    float *env_in, int64_t ld_env, xpa_stream_t stream) {
    if (n_envs <= 0 || act_dim < 1 || act_dim > kRolloutKMax || horizon <= 0 || hidden != 256 || ld < 256 || ld % 4 ||
        act < 0 || act > 2 || !z_actor || !z_critic || !w_actor || !b_actor || !w_critic || !b_critic || !cursor ||
        !buf_act || !buf_logp || !buf_val || !env_in || ld_env < act_dim)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)z_actor | (uintptr_t)z_critic | (uintptr_t)w_actor | (uintptr_t)w_critic) % 16)
        return (int)hipErrorInvalidValue;
    if ((dist == XPA_DIST_GAUSSIAN && !logstd) || (dist == XPA_DIST_CATEGORICAL && act_dim < 2) ||
        (dist != XPA_DIST_GAUSSIAN && dist != XPA_DIST_CATEGORICAL))
        return (int)hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((n_envs + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
#define XPA_K14(M_, A_)                                                                                          \
    hipLaunchKernelGGL((rollout_policy_head_kernel<M_, A_>), dim3(blocks), dim3(256), 0, s, n_envs, (int)act_dim, \
                       horizon, z_actor, z_critic, ld, slope, w_actor, b_actor, w_critic, b_critic, logstd, cursor,   \
                       seed, act_clip, buf_act, buf_logp, buf_val, env_in, ld_env, (float *)nullptr, SynthEnvArgs{})
    if (dist == XPA_DIST_GAUSSIAN) {
        if (act == 0) XPA_K14(0, 0);
        else if (act == 1) XPA_K14(0, 1);
        else XPA_K14(0, 2);
    } else {
        if (act == 0) XPA_K14(1, 0);
        else if (act == 1) XPA_K14(1, 1);
        else XPA_K14(1, 2);
    }
#undef XPA_K14
    return xpa_launch_status();
}

XPA_API int xpa_value_head(int act, int64_t n, int64_t hidden, int64_t ld, const float *z_critic, float slope,
                           const float *w_critic, const float *b_critic, float *v_out, xpa_stream_t stream) {
    if (n <= 0 || hidden != 256 || ld < 256 || ld % 4 || act < 0 || act > 2 || !z_critic || !w_critic ||
        !b_critic || !v_out || ((uintptr_t)z_critic | (uintptr_t)w_critic) % 16)
        return (int)hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((n + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
#define XPA_VH(A_)                                                                                                 \
    hipLaunchKernelGGL((rollout_policy_head_kernel<2, A_>), dim3(blocks), dim3(256), 0, s, n, 1, (int64_t)1,        \
                       z_critic, z_critic, ld, slope, w_critic, b_critic, w_critic, b_critic, (const float *)nullptr, \
                       (const xpa_cursor_t *)nullptr, 0u, 0.f, (float *)nullptr, (float *)nullptr, (float *)nullptr, \
                       (float *)nullptr, (int64_t)0, v_out, SynthEnvArgs{})
    if (act == 0) XPA_VH(0);
    else if (act == 1) XPA_VH(1);
    else XPA_VH(2);
#undef XPA_VH
    return xpa_launch_status();
}

XPA_API int xpa_store_column(const void *src, int64_t n, int64_t row_bytes, void *dst, int64_t horizon,
                             const xpa_cursor_t *cursor, xpa_stream_t stream) {
    if (n <= 0 || row_bytes <= 0 || row_bytes % 16 || horizon <= 0 || !src || !dst || !cursor ||
        ((uintptr_t)src | (uintptr_t)dst) % 16)
        return (int)hipErrorInvalidValue;
    const int64_t rv = row_bytes / 16;
    int64_t blocks = (n * rv + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(store_column_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const u4v *)src, n, rv, (u4v *)dst, horizon, cursor);
    return xpa_launch_status();
}

XPA_API int xpa_random_permutation(int64_t n, uint32_t seed, uint32_t counter, int64_t *out, xpa_stream_t stream) {
    if (n <= 0 || n > (1LL << 31) || !out) return (int)hipErrorInvalidValue;
    int h = 1;
    while ((1LL << (2 * h)) < n) ++h;
    hipLaunchKernelGGL(permutation_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, h,
                       seed, counter, out);
    return xpa_launch_status();
}

XPA_API int xpa_rollout_policy_head_synthbox(int act, int64_t n_envs, int64_t act_dim, int64_t horizon, int64_t hidden,
                                             int64_t ld, const float *z_actor, const float *z_critic, float slope,
                                             const float *w_actor, const float *b_actor, const float *w_critic,
                                             const float *b_critic, const float *logstd, const xpa_cursor_t *cursor,
                                             uint32_t seed, float act_clip, float *buf_act, float *buf_logp,
                                             float *buf_val, int64_t obs_dim, const float *wcat_t, uint32_t env_seed,
                                             int32_t max_episode_steps, float noise, float term_thresh,
                                             float reset_scale, float *state, int64_t ld_state, float *final_obs,
                                             float *rew, uint8_t *term, uint8_t *trunc, int32_t *ep_step,
                                             uint32_t *ep_index, float *ep_score, float *ep_last_score,
                                             int32_t *ep_last_len, xpa_stream_t stream) {
    if (n_envs <= 0 || act_dim < 1 || act_dim > kRolloutKMax || horizon <= 0 || hidden != 256 || ld < 256 || ld % 4 ||
        act < 0 || act > 2 || !z_actor || !z_critic || !w_actor || !b_actor || !w_critic || !b_critic || !cursor ||
        !logstd || !buf_act || !buf_logp || !buf_val)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)z_actor | (uintptr_t)z_critic | (uintptr_t)w_actor | (uintptr_t)w_critic) % 16)
        return (int)hipErrorInvalidValue;
    if (obs_dim < 1 || obs_dim > 64 || !wcat_t || !state || ld_state < obs_dim + act_dim || !final_obs || !rew ||
        !term || !trunc || !ep_step || !ep_index || !ep_score || !ep_last_score || !ep_last_len)
        return (int)hipErrorInvalidValue;
    SynthEnvArgs e{(int)obs_dim, env_seed, max_episode_steps, noise, term_thresh, reset_scale, state, ld_state,
                   final_obs, rew, term, trunc, ep_step, ep_index, ep_score, ep_last_score, ep_last_len, wcat_t};
    float *env_in = state + obs_dim;  // the action columns of the env's input rows (s | a)
    const unsigned blocks = (unsigned)((n_envs + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
#define XPA_K14E(A_)                                                                                              \
    hipLaunchKernelGGL((rollout_policy_head_kernel<0, A_, true>), dim3(blocks), dim3(256), 0, s, n_envs,           \
                       (int)act_dim, horizon, z_actor, z_critic, ld, slope, w_actor, b_actor, w_critic, b_critic,     \
                       logstd, cursor, seed, act_clip, buf_act, buf_logp, buf_val, env_in, ld_state, (float *)nullptr, \
                       e)
    if (act == 0) XPA_K14E(0);
    else if (act == 1) XPA_K14E(1);
    else XPA_K14E(2);
#undef XPA_K14E
    return xpa_launch_status();
}

// ---- K14F (r06) ------------------------------------------------------------------------------------
XPA_API int xpa_k14f_probe(int bits) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_k14f_probe), &bits, sizeof(int));
}

// Workspace of xpa_rollout_step_synthbox: f64 partials (returned, in doubles) and *n_tickets int32 tickets (zeroed once
// by the caller; every launch leaves them zero).  rms: with the obs_rms update.
XPA_API int64_t xpa_rollout_step_workspace(int64_t n_envs, int64_t obs_dim, int rms, int64_t *n_tickets) {
    if (n_envs <= 0 || obs_dim < 1 || obs_dim > 64 || !n_tickets) return -1;
    const int64_t blocks = (n_envs + 3) / 4, groups = (blocks + kPostGrp - 1) / kPostGrp;
    *n_tickets = (1 + groups) * kTicketStride;
    return (blocks + groups) * (3 + (rms ? 2 * obs_dim : 0));
}

// xpa_rollout_policy_head_synthbox and K8's deferred + normalised post step (xpa_rollout_post_deferred_norm, with
// obs_count non-null also the next step's obs_rms.update: xpa_rollout_post_deferred_norm_rms) in ONE launch (K14F).
// The post arguments mean what they mean there; slot_from_next (A2C's boot_from_reset): kept truncation rows are the
// env's next observation instead of its final one; part / tickets: xpa_rollout_step_workspace.
XPA_API int xpa_rollout_step_synthbox(
    int act, int64_t n_envs, int64_t act_dim, int64_t horizon, int64_t hidden, int64_t ld, const float *z_actor,
    const float *z_critic, float slope, const float *w_actor, const float *b_actor, const float *w_critic,
    const float *b_critic, const float *logstd, xpa_cursor_t *cursor, uint32_t seed, float act_clip, float *buf_act,
    float *buf_logp, float *buf_val, int64_t obs_dim, const float *wcat_t, uint32_t env_seed, int32_t max_episode_steps,
    float noise, float term_thresh, float reset_scale, float *state, int64_t ld_state, float *final_obs, float *rew,
    uint8_t *term, uint8_t *trunc, int32_t *ep_step, uint32_t *ep_index, float *ep_score, float *ep_last_score,
    int32_t *ep_last_len, float *slot_obs, int32_t *slot_t, int64_t n_slots, int32_t *overflow, int slot_from_next,
    float *obs_mean, float *obs_var, double *obs_count, float obs_clip, float *boot_norm, int64_t ld_norm,
    float *ret_mean, float *ret_var, double *ret_count, float *returns, float *buf_rew, float *buf_term,
    uint8_t *buf_closed, float *buf_boot, float gamma, int mask_returns, int use_rewnorm, float rew_range,
    int atari_lifeloss, double *part, int32_t *tickets, xpa_stream_t stream) {
    if (n_envs <= 0 || act_dim < 1 || act_dim > kRolloutKMax || horizon <= 0 || hidden != 256 || ld < 256 || ld % 4 ||
        act < 0 || act > 2 || !z_actor || !z_critic || !w_actor || !b_actor || !w_critic || !b_critic || !cursor ||
        !logstd || !buf_act || !buf_logp || !buf_val)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)z_actor | (uintptr_t)z_critic | (uintptr_t)w_actor | (uintptr_t)w_critic) % 16)
        return (int)hipErrorInvalidValue;
    if (obs_dim < 1 || obs_dim > 64 || !wcat_t || !state || ld_state < obs_dim + act_dim || !final_obs || !rew ||
        !term || !trunc || !ep_step || !ep_index || !ep_score || !ep_last_score || !ep_last_len)
        return (int)hipErrorInvalidValue;
    if (n_slots < 1 || n_slots > horizon || !slot_obs || !slot_t || !overflow || !obs_mean || !obs_var || !boot_norm ||
        ld_norm < obs_dim || !ret_mean || !ret_var || !ret_count || !returns || !buf_rew || !buf_term || !buf_closed ||
        !buf_boot || !part || !tickets || (n_envs + 3) / 4 > 0x7fffffff)
        return (int)hipErrorInvalidValue;
    SynthEnvArgs e{(int)obs_dim, env_seed, max_episode_steps, noise, term_thresh, reset_scale, state, ld_state,
                   final_obs, rew, term, trunc, ep_step, ep_index, ep_score, ep_last_score, ep_last_len, wcat_t};
    PostArgs pa{cursor, ret_mean, ret_var, ret_count, returns, buf_rew, buf_term, buf_closed, buf_boot, gamma, rew_range,
                obs_clip, mask_returns, use_rewnorm, atari_lifeloss, slot_from_next, (int)n_slots, slot_obs, slot_t,
                overflow, obs_mean, obs_var, obs_count, boot_norm, ld_norm, part, (unsigned *)tickets};
    float *env_in = state + obs_dim;
    const unsigned blocks = (unsigned)((n_envs + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
#define XPA_K14F(A_)                                                                                              \
    hipLaunchKernelGGL((rollout_policy_head_kernel<0, A_, true, true>), dim3(blocks), dim3(256), 0, s, n_envs,     \
                       (int)act_dim, horizon, z_actor, z_critic, ld, slope, w_actor, b_actor, w_critic, b_critic,     \
                       logstd, cursor, seed, act_clip, buf_act, buf_logp, buf_val, env_in, ld_state, (float *)nullptr, \
                       e, pa)
    if (act == 0) XPA_K14F(0);
    else if (act == 1) XPA_K14F(1);
    else XPA_K14F(2);
#undef XPA_K14F
    return xpa_launch_status();
}

// ---- K32 -------------------------------------------------------------------------------------------
XPA_API int64_t xpa_small_rollout_lds_floats(int64_t n_envs, int64_t d_in, int64_t h0, int64_t h1, int64_t h2,
                                             int64_t k) {
    if (n_envs <= 0 || n_envs > 256 || d_in <= 0 || d_in > 32 || h0 <= 0 || h0 > 64 || h1 <= 0 || h1 > 64 ||
        h2 <= 0 || h2 > 64 || k <= 0 || k > 16)
        return -1;
    return ro_layout((int)n_envs, (int)d_in, (int)h0, (int)h1, (int)h2, (int)k).total;
}

XPA_API int xpa_small_rollout_cartpole(const XpaSmallRolloutArgs *a, xpa_stream_t stream) {
    if (!a || a->n_envs <= 0 || a->n_envs > 256 || a->horizon <= 0 || a->steps <= 0 || a->d_in != 4 ||
        (a->h0 != 32 && a->h0 != 64) || (a->h1 != 32 && a->h1 != 64) || (a->h2 != 32 && a->h2 != 64) || a->k != 2 ||
        a->act_code < 0 || a->act_code > 2 || a->n_slots < 1 || a->n_slots > a->horizon || a->max_episode_steps <= 0 ||
        a->ld_norm < a->d_in || a->ld_obs < 4 || a->ld_act < 2 || a->ld_boot < a->d_in)
        return (int)hipErrorInvalidValue;
    if (!a->W0 || !a->b0 || !a->W1 || !a->b1 || !a->W2 || !a->b2 || !a->Wa || !a->ba || !a->Wc || !a->bc ||
        !a->obs_mean || !a->obs_var || !a->obs_count || !a->obs_norm || !a->buf_obs || !a->buf_act || !a->buf_logp ||
        !a->buf_val || !a->buf_rew || !a->buf_term || !a->buf_closed || !a->buf_boot || !a->act_in || !a->env_state ||
        !a->env_obs || !a->final_obs || !a->env_rew || !a->env_term || !a->env_trunc || !a->ep_step || !a->ep_index ||
        !a->ep_score || !a->ep_last_score || !a->ep_last_len || !a->returns || !a->ret_mean || !a->ret_var ||
        !a->ret_count || !a->slot_obs || !a->slot_t || !a->overflow || !a->boot_norm || !a->cursor)
        return (int)hipErrorInvalidValue;
    const int64_t lf = xpa_small_rollout_lds_floats(a->n_envs, a->d_in, a->h0, a->h1, a->h2, a->k);
    if (lf < 0 || lf > kRoLdsMax) return (int)hipErrorInvalidValue;
    const size_t bytes = (size_t)lf * sizeof(float);
    hipStream_t s = (hipStream_t)stream;
#define XPA_RO_LAUNCH(ACT, H0) \
    hipLaunchKernelGGL((small_rollout_cartpole_kernel<ACT, H0>), dim3(1), dim3(kRoThreads), bytes, s, *a)
    if (a->h0 == 64) {
        if (a->act_code == 0) XPA_RO_LAUNCH(0, 64);
        else if (a->act_code == 1) XPA_RO_LAUNCH(1, 64);
        else XPA_RO_LAUNCH(2, 64);
    } else {
        if (a->act_code == 0) XPA_RO_LAUNCH(0, 32);
        else if (a->act_code == 1) XPA_RO_LAUNCH(1, 32);
        else XPA_RO_LAUNCH(2, 32);
    }
#undef XPA_RO_LAUNCH
    return xpa_launch_status();
}
