// K13 — the representation's first layer, Linear(d_in, 256) + activation with a small d_in (the
// observation width: 17 for the C2 MuJoCo shape), forward and backward as streaming kernels (gfx950).
//
// Reference: Basic_MLP's first mlp_block (xuance/torch/representations/mlp.py:21-51,
// xuance/torch/utils/layers.py:8-24); forward in policy(obs) and backward in loss.backward()
// (ppoclip_learner.py:30-46).  With K = d_in <= 64 the GEMM has ~17 FMAs per output element, so the
// layer is bound by HBM (writing / re-reading the [B, 256] activations), not by the matrix cores.
//
//   forward : h[b, c] = act(sum_k x[b, k] W[c, k] + bias[c])      (writes h: 1 KiB per row)
//   backward: dz = g * act'(h);  dW[c, k] = sum_b dz[b, c] x[b, k];  db[c] = sum_b dz[b, c]
//             (reads g and h: 2 KiB per row; dz itself is never stored — nothing below the first
//             layer needs it)
// Mapping: 256 threads, thread t owns output column t (its d_in weights / accumulators in registers);
// a block walks 64-row tiles (grid-stride); the tile's x rows are staged in LDS and read as
// wave-uniform broadcasts; h / g rows are read and written as whole coalesced 1-KiB rows.
#include "xpa_common.h"

namespace {

constexpr int kCols = 256;
constexpr int kTile = 64;
constexpr int kMaxIn = 64;
constexpr int kFwdGrid = 1024;
constexpr int kBwdGrid = 256;

template <int ACT>
__device__ __forceinline__ float act_f(float z, float slope) {
    if (ACT == 1) return z > 0.f ? z : z * slope;
    if (ACT == 2) return tanhf(z);
    return z;
}

template <int ACT>
__device__ __forceinline__ float act_g(float h, float slope) {
    if (ACT == 1) return h > 0.f ? 1.f : slope;
    if (ACT == 2) return 1.0f - h * h;
    return 1.f;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// IDX: the rows are x[idx[r]] of the full rollout buffer (n_rows rows; an index outside [0, n_rows) gives a zero row
// and adds nothing to the moments), i.e. K4's minibatch gather folded into the staging of the x tile, and with
// adv_partials the K4 advantage moments of each 64-row tile (f64 (sum, sum of squares), thread t <-> row t and
// xpa_block_sum: K4's partials bit for bit).  Only the 64-row tile form takes IDX.
// NT: h stored non-temporally (the default); false (xpa_thin_probe bit 1, r04 A/B): plain stores, so the update's h
// may stay in the caches for the head launches and K41 that read it next
template <int ACT, int DMAX, int TILE, bool IDX = false, bool NT = true>
__global__ __launch_bounds__(256) void thin_fwd_kernel(const float *__restrict__ x, int64_t ldx, int64_t rows, int din,
                                                       const float *__restrict__ W, const float *__restrict__ bias,
                                                       float slope, float *__restrict__ h, int64_t ldh,
                                                       const int64_t *__restrict__ idx = nullptr, int64_t n_rows = 0,
                                                       const float *__restrict__ adv = nullptr,
                                                       double *__restrict__ adv_partials = nullptr,
                                                       float *__restrict__ x_out = nullptr,
                                                       unsigned *__restrict__ hsign = nullptr) {
    // the staged x tile as row pairs: element (r, k) at ((r >> 1) DMAX + k) 2 + (r & 1), so one float4 broadcast
    // read holds features k, k + 1 of rows r, r + 1 and each v_pk_fma_f32 runs the two rows' chains (r04: one
    // fmaf chain per row — 45 instructions per row and wave — kept the kernel VALU-issue bound); every chain is
    // still the same k-ascending fmaf sequence, so h is bit for bit the one-row form's
    static_assert(TILE % 2 == 0 && DMAX % 2 == 0, "row pairs, feature pairs");
    __shared__ __attribute__((aligned(16))) float s_x[TILE * DMAX];
    __shared__ unsigned long long s_ball[IDX ? TILE * 4 : 1];   // hsign: each wave's h > 0 ballot per row
    __shared__ int64_t s_src[IDX ? TILE : 1];
    __shared__ double s_red[4];
    const int t = threadIdx.x;
    float w[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) w[k] = k < din ? W[t * din + k] : 0.f;
    const float bc = bias[t];
    const int64_t ntiles = (rows + TILE - 1) / TILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * TILE;
        __syncthreads();
        if (IDX) {
            if (t < TILE) {
                const int64_t sr = r0 + t < rows ? idx[r0 + t] : -1;
                s_src[t] = (sr >= 0 && sr < n_rows) ? sr : -1;
            }
            __syncthreads();
        }
        // zero-padded columns din..DMAX-1 stay 0 from this loop's (r, k < DMAX) writes
        float av = 0.f;
        if constexpr (IDX) {
            // every load of the tile issued before the first use (clamped addresses, validity by select; r02: the
            // loads under the validity branch each waited at the join — one round trip per element and one for adv)
            constexpr int kPer = (TILE * DMAX + 255) / 256;
            float v[kPer];
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int i = t + 256 * u;
                const int r = i < TILE * DMAX ? i / DMAX : 0, k = i - (i / DMAX) * DMAX;
                const int64_t sr = s_src[r];
                const bool ok = i < TILE * DMAX && k < din && sr >= 0;
                v[u] = x[ok ? sr * ldx + k : 0];
                v[u] = ok ? v[u] : 0.f;
            }
            const int64_t sa = t < TILE ? s_src[t] : -1;
            if (adv_partials) {
                av = adv[sa >= 0 ? sa : 0];
                av = sa >= 0 ? av : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int i = t + 256 * u;
                if (i < TILE * DMAX) {
                    const int r = i / DMAX, k = i - r * DMAX;
                    s_x[((r >> 1) * DMAX + k) * 2 + (r & 1)] = v[u];
                    if (x_out && k < din && r0 + r < rows) x_out[(r0 + r) * din + k] = v[u];  // the gathered rows
                }
            }
        } else {
            for (int i = t; i < TILE * DMAX; i += 256) {
                const int r = i / DMAX, k = i - r * DMAX;
                s_x[((r >> 1) * DMAX + k) * 2 + (r & 1)] = (k < din && r0 + r < rows) ? x[(r0 + r) * ldx + k] : 0.f;
            }
        }
        if (IDX && adv_partials) {  // K4's moments of this tile (thread t <-> row t)
            double sm = 0.0, q = 0.0;
            {
                const double a = (double)av;   // 0 for an invalid row: adds nothing, as before
                sm = a;
                q = a * a;
            }
            sm = xpa_block_sum(sm, s_red, 4);
            q = xpa_block_sum(q, s_red, 4);
            if (t == 0) {
                adv_partials[2 * tile] = sm;
                adv_partials[2 * tile + 1] = q;
            }
        }
        if (IDX && !h) continue;  // gather-only form (K16X forms h itself): the rows and the moments
        __syncthreads();
        const int nr = (int)min((int64_t)TILE, rows - r0);
        for (int r = 0; r < nr; r += 2) {   // rows r, r + 1 (a row past the tile's end is staged as zeros)
            const float4 *xp = reinterpret_cast<const float4 *>(s_x + (r >> 1) * DMAX * 2);
            f2 acc = {0.f, 0.f};
#pragma unroll
            for (int k = 0; k < DMAX; k += 2) {
                const float4 xv = xp[k >> 1];   // (x[r][k], x[r + 1][k], x[r][k + 1], x[r + 1][k + 1])
                acc = __builtin_elementwise_fma(f2{xv.x, xv.y}, f2{w[k], w[k]}, acc);
                acc = __builtin_elementwise_fma(f2{xv.z, xv.w}, f2{w[k + 1], w[k + 1]}, acc);
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                if (e == 1 && r + 1 >= nr) break;
                const float hv = act_f<ACT>(acc[e] + bc, slope);
                if constexpr (NT) __builtin_nontemporal_store(hv, h + (r0 + r + e) * ldh + t);
                else h[(r0 + r + e) * ldh + t] = hv;
                if (IDX && hsign != nullptr) {
                    const unsigned long long bl = __ballot(hv > 0.f);
                    if ((t & 63) == 0) s_ball[(r + e) * 4 + (t >> 6)] = bl;
                }
            }
        }
        if (IDX && hsign != nullptr) {
            // the sign bits in K42S's lane order: byte b of a row's 32 bytes, bit j = h[row, 32 j + b] > 0 (column
            // 32 j + b is lane 32 (j & 1) + b of wave j >> 1); thread t writes words 2 (t & 3), + 1 of row t >> 2
            __syncthreads();
            const int r = t >> 2;
            if (r < nr) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int d = 2 * (t & 3) + u;   // bytes 4 d .. 4 d + 3
                    unsigned word = 0u;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const unsigned v = (unsigned)(s_ball[r * 4 + (j >> 1)] >> (32 * (j & 1) + 4 * d)) & 0xFu;
                        word |= ((v & 1u) | ((v & 2u) << 7) | ((v & 4u) << 14) | ((v & 8u) << 21)) << j;
                    }
                    hsign[(r0 + r) * 8 + d] = word;
                }
            }
        }
    }
}

// Rollout form with the observation normalisation fused in (K5c + K13): the raw observation rows are
// normalised while the x tile is staged — clip((x - mean) / (sqrt(var) + 1e-8)), xpa_obs_normalize's
// arithmetic — and the normalised rows are also written to `xn` (the policy input) and into the
// rollout buffer column cursor.ptr of `col` ([rows, T, din] at col_ld floats per row).  8-row tiles.
template <int ACT, int DMAX>
__global__ __launch_bounds__(256) void thin_fwd_norm_kernel(const float *__restrict__ x, int64_t ldx, int64_t rows,
                                                            int din, const float *__restrict__ W,
                                                            const float *__restrict__ bias, float slope,
                                                            float *__restrict__ h, int64_t ldh,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ var, float clip,
                                                            float *__restrict__ xn, int64_t ldn,
                                                            float *__restrict__ col, int64_t col_ld,
                                                            const xpa_cursor_t *__restrict__ cursor, int h_nt) {
    constexpr int TILE = 8;
    constexpr int kPad = DMAX + 4;
    __shared__ __attribute__((aligned(16))) float s_x[TILE * kPad];
    const int t = threadIdx.x;
    float w[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) w[k] = k < din ? W[t * din + k] : 0.f;
    const float bc = bias[t];
    const int64_t coff = col ? (int64_t)cursor->ptr * din : 0;
    const int64_t ntiles = (rows + TILE - 1) / TILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * TILE;
        __syncthreads();
        for (int i = t; i < TILE * DMAX; i += 256) {
            // loads unconditional from clamped addresses (under the validity branch hipcc waited for them at the
            // join, after the weight loads: two serial round trips per tile)
            const int r = i / DMAX, k = i - r * DMAX;
            const bool ok = k < din && r0 + r < rows;
            const int kc = k < din ? k : 0;
            const int64_t rc = r0 + r < rows ? r0 + r : r0;
            const float xv = x[rc * ldx + kc], mv = mean[kc], vv = var[kc];
            float y = 0.f;
            if (ok) {
                const float sd = sqrtf(vv);
                y = (xv - mv) / (sd + 1e-8f);
                y = fminf(fmaxf(y, -clip), clip);
                xn[(r0 + r) * ldn + k] = y;
                if (col) col[(r0 + r) * col_ld + coff + k] = y;
            }
            s_x[r * kPad + k] = y;
        }
        __syncthreads();
        const int nr = (int)min((int64_t)TILE, rows - r0);
        for (int r = 0; r < nr; ++r) {
            const float *xr = s_x + r * kPad;
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < DMAX; k += 4) {
                const float4 xv = *reinterpret_cast<const float4 *>(xr + k);
                acc = fmaf(xv.x, w[k], acc);
                acc = fmaf(xv.y, w[k + 1], acc);
                acc = fmaf(xv.z, w[k + 2], acc);
                acc = fmaf(xv.w, w[k + 3], acc);
            }
            // non-temporal by default; xpa_thin_probe bit 2 (r05 A/B): plain stores, so the paired hidden GEMM (K40R,
            // XCD-mapped rows) might read h from L2 — measured no faster (profiles/r05/r05r2_*: 5.77 vs 5.61 ms rollout)
            const float hv = act_f<ACT>(acc + bc, slope);
            if (h_nt) __builtin_nontemporal_store(hv, h + (r0 + r) * ldh + t);
            else h[(r0 + r) * ldh + t] = hv;
        }
    }
}

// 1024 threads = 4 groups of 256 (group = one 64-row tile at a time, thread = column), 8 rows of g / h
// in flight per thread; the groups' accumulators are combined through LDS (fixed order) at the end.
constexpr int kBwdGroups = 4;
constexpr int kBwdU = 8;

template <int ACT, int DMAX, bool IDX = false>
__global__ __launch_bounds__(1024) void thin_bwd_kernel(const float *__restrict__ g, int64_t ldg,
                                                        const float *__restrict__ h, int64_t ldh, int64_t rows,
                                                        const float *__restrict__ x, int64_t ldx, int din, float slope,
                                                        float *__restrict__ partial_dw, float *__restrict__ partial_db,
                                                        const int64_t *__restrict__ idx = nullptr, int64_t n_rows = 0) {
    constexpr int kPad = DMAX + 4;
    constexpr int kXs = kTile * kPad;                                        // one group's x tile
    constexpr int kLds = kBwdGroups * kXs > kCols * (DMAX + 1) ? kBwdGroups * kXs : kCols * (DMAX + 1);
    __shared__ __attribute__((aligned(16))) float s_buf[kLds];
    const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
    float *s_x = s_buf + grp * kXs;
    float acc[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) acc[k] = 0.f;
    float accb = 0.f;
    const int64_t ntiles = (rows + kTile - 1) / kTile;
    for (int64_t base = (int64_t)blockIdx.x * kBwdGroups; base < ntiles; base += (int64_t)gridDim.x * kBwdGroups) {
        const int64_t tile = base + grp;  // uniform trip count for the whole block (barriers)
        const int64_t r0 = tile * kTile;
        __syncthreads();
        if (tile < ntiles) {
            for (int i = t; i < kTile * DMAX; i += 256) {
                const int r = i / DMAX, k = i - r * DMAX;
                if (IDX) {  // the minibatch row r of the full buffer (K4's gather folded in; out of range: zero row)
                    const int64_t sr = r0 + r < rows ? idx[r0 + r] : -1;
                    s_x[r * kPad + k] = (k < din && sr >= 0 && sr < n_rows) ? x[sr * ldx + k] : 0.f;
                } else {
                    s_x[r * kPad + k] = (k < din && r0 + r < rows) ? x[(r0 + r) * ldx + k] : 0.f;
                }
            }
        }
        __syncthreads();
        if (tile >= ntiles) continue;
        const int nr = (int)min((int64_t)kTile, rows - r0);
        int r = 0;
        for (; r + kBwdU <= nr; r += kBwdU) {
            float gv[kBwdU], hv[kBwdU];
#pragma unroll
            for (int u = 0; u < kBwdU; ++u) {
                gv[u] = __builtin_nontemporal_load(g + (r0 + r + u) * ldg + t);
                hv[u] = __builtin_nontemporal_load(h + (r0 + r + u) * ldh + t);
            }
#pragma unroll
            for (int u = 0; u < kBwdU; ++u) {
                const float dz = gv[u] * act_g<ACT>(hv[u], slope);
                accb += dz;
                const float *xr = s_x + (r + u) * kPad;
#pragma unroll
                for (int k = 0; k < DMAX; k += 4) {
                    const float4 xv = *reinterpret_cast<const float4 *>(xr + k);
                    acc[k] = fmaf(dz, xv.x, acc[k]);
                    acc[k + 1] = fmaf(dz, xv.y, acc[k + 1]);
                    acc[k + 2] = fmaf(dz, xv.z, acc[k + 2]);
                    acc[k + 3] = fmaf(dz, xv.w, acc[k + 3]);
                }
            }
        }
        for (; r < nr; ++r) {
            const float dz = g[(r0 + r) * ldg + t] * act_g<ACT>(h[(r0 + r) * ldh + t], slope);
            accb += dz;
            const float *xr = s_x + r * kPad;
#pragma unroll
            for (int k = 0; k < DMAX; ++k) acc[k] = fmaf(dz, xr[k], acc[k]);
        }
    }
    // combine groups 1..3 into group 0 (fixed order), through LDS [256][DMAX + 1]
    for (int src = 1; src < kBwdGroups; ++src) {
        __syncthreads();
        if (grp == src) {
#pragma unroll
            for (int k = 0; k < DMAX; ++k) s_buf[t * (DMAX + 1) + k] = acc[k];
            s_buf[t * (DMAX + 1) + DMAX] = accb;
        }
        __syncthreads();
        if (grp == 0) {
#pragma unroll
            for (int k = 0; k < DMAX; ++k) acc[k] += s_buf[t * (DMAX + 1) + k];
            accb += s_buf[t * (DMAX + 1) + DMAX];
        }
    }
    if (grp != 0) return;
    // partial row layout = the weight layout [256, din] (row-major), so a column sum over the
    // partials lands directly in W.grad
    float *pw = partial_dw + (int64_t)blockIdx.x * kCols * din + (int64_t)t * din;
#pragma unroll
    for (int k = 0; k < DMAX; ++k)
        if (k < din) pw[k] = acc[k];
    partial_db[(int64_t)blockIdx.x * kCols + t] = accb;
}

template <int ACT, int TILE>
void launch_fwd_t(int dmax, dim3 grid, hipStream_t s, const float *x, int64_t ldx, int64_t rows, int din,
                  const float *W, const float *b, float slope, float *h, int64_t ldh) {
#define XPA_FWD(D_) \
    hipLaunchKernelGGL((thin_fwd_kernel<ACT, D_, TILE>), grid, dim3(256), 0, s, x, ldx, rows, din, W, b, slope, h, ldh)
    if (dmax == 8) XPA_FWD(8);
    else if (dmax == 20) XPA_FWD(20);
    else if (dmax == 32) XPA_FWD(32);
    else XPA_FWD(64);
#undef XPA_FWD
}

// 64-row tiles for update-sized batches; 8-row tiles when fewer than 1024 x 64 rows (e.g. the rollout's
// 4096 envs) so the grid still covers the chip.
template <int ACT>
void launch_fwd(int dmax, hipStream_t s, const float *x, int64_t ldx, int64_t rows, int din, const float *W,
                const float *b, float slope, float *h, int64_t ldh) {
    if (rows >= (int64_t)kTile * kFwdGrid) {
        launch_fwd_t<ACT, kTile>(dmax, dim3(kFwdGrid), s, x, ldx, rows, din, W, b, slope, h, ldh);
    } else {
        const int64_t tiles = (rows + 7) / 8;
        launch_fwd_t<ACT, 8>(dmax, dim3((unsigned)(tiles < kFwdGrid ? tiles : kFwdGrid)), s, x, ldx, rows, din, W, b,
                             slope, h, ldh);
    }
}

template <int ACT>
void launch_bwd(int dmax, dim3 grid, hipStream_t s, const float *g, int64_t ldg, const float *h, int64_t ldh,
                int64_t rows, const float *x, int64_t ldx, int din, float slope, float *pdw, float *pdb) {
#define XPA_BWD(D_) \
    hipLaunchKernelGGL((thin_bwd_kernel<ACT, D_>), grid, dim3(1024), 0, s, g, ldg, h, ldh, rows, x, ldx, din, slope, pdw, pdb)
    if (dmax == 8) XPA_BWD(8);
    else if (dmax == 20) XPA_BWD(20);
    else if (dmax == 32) XPA_BWD(32);
    else XPA_BWD(64);
#undef XPA_BWD
}

int dmax_for(int din) { return din <= 8 ? 8 : din <= 20 ? 20 : din <= 32 ? 32 : 64; }

}  // namespace

// diagnostics / A-B (tools): bit 1 = the sign gather form with plain (not non-temporal) h stores
static int g_thin_probe = 0;
XPA_API int xpa_thin_probe(int mask) {
    g_thin_probe = mask;
    return 0;
}

XPA_API int64_t xpa_thin_bwd_num_partials(int64_t rows) {
    const int64_t blocks = ((rows + kTile - 1) / kTile + 3) / 4;  // 4 tiles per block-iteration
    return blocks < kBwdGrid ? (blocks > 0 ? blocks : 1) : kBwdGrid;
}

XPA_API int xpa_thin_linear_act_fwd(int act, const float *x, int64_t ldx, int64_t rows, int64_t d_in, int64_t d_out,
                                    const float *w, const float *b, float slope, float *h, int64_t ldh,
                                    xpa_stream_t stream) {
    if (rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 2 || !x || !w || !b || !h ||
        ldx < d_in || ldh < d_out)
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int dm = dmax_for((int)d_in);
    if (act == 0) launch_fwd<0>(dm, s, x, ldx, rows, (int)d_in, w, b, slope, h, ldh);
    else if (act == 1) launch_fwd<1>(dm, s, x, ldx, rows, (int)d_in, w, b, slope, h, ldh);
    else launch_fwd<2>(dm, s, x, ldx, rows, (int)d_in, w, b, slope, h, ldh);
    return xpa_launch_status();
}

XPA_API int xpa_thin_linear_act_bwd(int act, const float *g, int64_t ldg, const float *h, int64_t ldh, int64_t rows,
                                    const float *x, int64_t ldx, int64_t d_in, int64_t d_out, float slope,
                                    float *partial_dw, float *partial_db, xpa_stream_t stream) {
    if (rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 2 || !g || !h || !x ||
        !partial_dw || !partial_db || ldg < d_out || ldh < d_out || ldx < d_in)
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_thin_bwd_num_partials(rows));
    hipStream_t s = (hipStream_t)stream;
    const int dm = dmax_for((int)d_in);
    if (act == 0) launch_bwd<0>(dm, grid, s, g, ldg, h, ldh, rows, x, ldx, (int)d_in, slope, partial_dw, partial_db);
    else if (act == 1) launch_bwd<1>(dm, grid, s, g, ldg, h, ldh, rows, x, ldx, (int)d_in, slope, partial_dw, partial_db);
    else launch_bwd<2>(dm, grid, s, g, ldg, h, ldh, rows, x, ldx, (int)d_in, slope, partial_dw, partial_db);
    return xpa_launch_status();
}

XPA_API int xpa_thin_linear_act_fwd_norm(int act, const float *x, int64_t ldx, int64_t rows, int64_t d_in,
                                         int64_t d_out, const float *w, const float *b, float slope, float *h,
                                         int64_t ldh, const float *mean, const float *var, float clip, float *xn,
                                         int64_t ldn, float *col, int64_t col_ld, const xpa_cursor_t *cursor,
                                         xpa_stream_t stream) {
    if (rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 2 || !x || !w || !b || !h ||
        !mean || !var || !xn || ldx < d_in || ldh < d_out || ldn < d_in || (col && (!cursor || col_ld < d_in)))
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int64_t tiles = (rows + 7) / 8;
    const dim3 grid((unsigned)(tiles < kFwdGrid ? tiles : kFwdGrid));
    const int dm = dmax_for((int)d_in);
#define XPA_FWDN(A_, D_)                                                                                            \
    hipLaunchKernelGGL((thin_fwd_norm_kernel<A_, D_>), grid, dim3(256), 0, s, x, ldx, rows, (int)d_in, w, b, slope, h, \
                       ldh, mean, var, clip, xn, ldn, col, col_ld, cursor, (g_thin_probe & 2) != 0 ? 0 : 1)
#define XPA_FWDN_D(A_)              \
    if (dm == 8) XPA_FWDN(A_, 8);   \
    else if (dm == 20) XPA_FWDN(A_, 20); \
    else if (dm == 32) XPA_FWDN(A_, 32); \
    else XPA_FWDN(A_, 64);
    if (act == 0) { XPA_FWDN_D(0) }
    else if (act == 1) { XPA_FWDN_D(1) }
    else { XPA_FWDN_D(2) }
#undef XPA_FWDN_D
#undef XPA_FWDN
    return xpa_launch_status();
}

XPA_API int xpa_thin_linear_act_fwd_gather(int act, const float *x, int64_t ldx, int64_t n_rows, const int64_t *idx,
                                           int64_t rows, int64_t d_in, int64_t d_out, const float *w, const float *b,
                                           float slope, float *h, int64_t ldh, const float *adv, double *adv_partials,
                                           float *x_out, xpa_stream_t stream) {
    if (rows <= 0 || n_rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 2 || !x || !idx ||
        !w || !b || (!h && !x_out) || ldx < d_in || (h && ldh < d_out) || (adv_partials && !adv))
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int64_t tiles = (rows + kTile - 1) / kTile;
    const dim3 grid((unsigned)(tiles < kFwdGrid ? tiles : kFwdGrid));
    const int dm = dmax_for((int)d_in);
#define XPA_FWDG(A_, D_)                                                                                             \
    hipLaunchKernelGGL((thin_fwd_kernel<A_, D_, kTile, true>), grid, dim3(256), 0, s, x, ldx, rows, (int)d_in, w, b,   \
                       slope, h, ldh, idx, n_rows, adv, adv_partials, x_out)
#define XPA_FWDG_D(A_)                 \
    if (dm == 8) XPA_FWDG(A_, 8);      \
    else if (dm == 20) XPA_FWDG(A_, 20); \
    else if (dm == 32) XPA_FWDG(A_, 32); \
    else XPA_FWDG(A_, 64);
    if (act == 0) { XPA_FWDG_D(0) }
    else if (act == 1) { XPA_FWDG_D(1) }
    else { XPA_FWDG_D(2) }
#undef XPA_FWDG_D
#undef XPA_FWDG
    return xpa_launch_status();
}

// the gather form writing h and its sign bits (h_sign: 32 bytes per row, byte b bit j = h[row, 32 j + b] > 0, the
// layout xpa_s3_gemm_trunk_bwd_sign reads); h and h_sign required, act 0 / 1 (the bits carry LeakyReLU's act')
XPA_API int xpa_thin_linear_act_fwd_gather_sign(int act, const float *x, int64_t ldx, int64_t n_rows,
                                                const int64_t *idx, int64_t rows, int64_t d_in, int64_t d_out,
                                                const float *w, const float *b, float slope, float *h, int64_t ldh,
                                                const float *adv, double *adv_partials, float *x_out,
                                                unsigned *h_sign, xpa_stream_t stream) {
    if (rows <= 0 || n_rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 1 || !x || !idx ||
        !w || !b || !h || !h_sign || ldx < d_in || ldh < d_out || (adv_partials && !adv))
        return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const int64_t tiles = (rows + kTile - 1) / kTile;
    const dim3 grid((unsigned)(tiles < kFwdGrid ? tiles : kFwdGrid));
    const int dm = dmax_for((int)d_in);
#define XPA_FWDG(A_, D_)                                                                                             \
    if (g_thin_probe & 1)                                                                                            \
        hipLaunchKernelGGL((thin_fwd_kernel<A_, D_, kTile, true, false>), grid, dim3(256), 0, s, x, ldx, rows,        \
                           (int)d_in, w, b, slope, h, ldh, idx, n_rows, adv, adv_partials, x_out, h_sign);           \
    else                                                                                                             \
        hipLaunchKernelGGL((thin_fwd_kernel<A_, D_, kTile, true>), grid, dim3(256), 0, s, x, ldx, rows, (int)d_in, w, \
                           b, slope, h, ldh, idx, n_rows, adv, adv_partials, x_out, h_sign)
#define XPA_FWDG_D(A_)                 \
    if (dm == 8) XPA_FWDG(A_, 8);      \
    else if (dm == 20) XPA_FWDG(A_, 20); \
    else if (dm == 32) XPA_FWDG(A_, 32); \
    else XPA_FWDG(A_, 64);
    if (act == 0) { XPA_FWDG_D(0) }
    else { XPA_FWDG_D(1) }
#undef XPA_FWDG_D
#undef XPA_FWDG
    return xpa_launch_status();
}

XPA_API int xpa_thin_linear_act_bwd_gather(int act, const float *g, int64_t ldg, const float *h, int64_t ldh,
                                           int64_t rows, const float *x, int64_t ldx, int64_t n_rows,
                                           const int64_t *idx, int64_t d_in, int64_t d_out, float slope,
                                           float *partial_dw, float *partial_db, xpa_stream_t stream) {
    if (rows <= 0 || n_rows <= 0 || d_in < 1 || d_in > kMaxIn || d_out != kCols || act < 0 || act > 2 || !g || !h ||
        !x || !idx || !partial_dw || !partial_db || ldg < d_out || ldh < d_out || ldx < d_in)
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)xpa_thin_bwd_num_partials(rows));
    hipStream_t s = (hipStream_t)stream;
    const int dm = dmax_for((int)d_in);
#define XPA_BWDG(A_, D_)                                                                                            \
    hipLaunchKernelGGL((thin_bwd_kernel<A_, D_, true>), grid, dim3(1024), 0, s, g, ldg, h, ldh, rows, x, ldx,         \
                       (int)d_in, slope, partial_dw, partial_db, idx, n_rows)
#define XPA_BWDG_D(A_)                 \
    if (dm == 8) XPA_BWDG(A_, 8);      \
    else if (dm == 20) XPA_BWDG(A_, 20); \
    else if (dm == 32) XPA_BWDG(A_, 32); \
    else XPA_BWDG(A_, 64);
    if (act == 0) { XPA_BWDG_D(0) }
    else if (act == 1) { XPA_BWDG_D(1) }
    else { XPA_BWDG_D(2) }
#undef XPA_BWDG_D
#undef XPA_BWDG
    return xpa_launch_status();
}
