// K10 — activation backward fused with the bias-gradient column sums of an MLP layer (gfx950).
//
// Replaces, in the learner's backward through the actor-critic (PPOCLIP_Learner.update's
// loss.backward(), xuance/torch/learners/policy_gradient/ppoclip_learner.py:46, through the
// mlp_block Linear -> activation layers of xuance/torch/utils/layers.py:8-24), the two torch passes
// over each [B, C] hidden activation: the activation backward (dz = dh * act'(h)) and the bias
// gradient reduction (db = sum_b dz).  One pass reads dh and h, writes dz (may alias dh) and per-block
// column partial sums; xpa_colsum_finalize reduces the partials (fixed order) into db.
// act: 0 = identity (output layers: only the column sums), 1 = LeakyReLU/ReLU with `slope`
// (the mask is taken from the activation OUTPUT h: h > 0 <=> z > 0 for slope >= 0), 2 = tanh (1 - h^2).
// HBM-bound: 12 B per element (dh, h read; dz written) + C*4 B per 256 rows of partials.
#include "xpa_common.h"
#include "loss_finalize.h"

namespace {

constexpr int kRowsPerBlock = 64;  // 1024 blocks at B = 65 536: ~4 blocks per CU to hide HBM latency

template <int ACT>
__device__ __forceinline__ float act_grad(float dh, float h, float slope) {
    if (ACT == 1) return h > 0.f ? dh : dh * slope;
    if (ACT == 2) return dh * (1.0f - h * h);
    return dh;
}

// C % 4 == 0: each thread owns 4 consecutive columns of its row group (16-B accesses).
// dh and dz may alias (in-place): no __restrict__ on them.
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd_colsum_vec4(const float *dh, const float *__restrict__ h, int64_t B,
                                                           int C, float slope, float *dz,
                                                           float *__restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) float4 s_acc[];  // [groups][C/4]
    const int cq = C / 4;                                            // <= 256 (checked by the launcher)
    const int groups = 256 / cq;
    const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
    const int64_t r1 = r0 + kRowsPerBlock < B ? r0 + kRowsPerBlock : B;
    const int c4 = threadIdx.x % cq, g = threadIdx.x / cq;
    if (g < groups) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int64_t r = r0 + g; r < r1; r += groups) {
            const int64_t off = r * C + 4 * c4;
            float4 d = *reinterpret_cast<const float4 *>(dh + off);
            if (ACT != 0) {
                const float4 hv = *reinterpret_cast<const float4 *>(h + off);
                d.x = act_grad<ACT>(d.x, hv.x, slope);
                d.y = act_grad<ACT>(d.y, hv.y, slope);
                d.z = act_grad<ACT>(d.z, hv.z, slope);
                d.w = act_grad<ACT>(d.w, hv.w, slope);
                if (dz) *reinterpret_cast<float4 *>(dz + off) = d;
            }
            acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
        }
        s_acc[g * cq + c4] = acc;
    }
    __syncthreads();
    for (int c4 = threadIdx.x; c4 < cq; c4 += 256) {
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int g = 0; g < groups; ++g) {
            const float4 a = s_acc[g * cq + c4];
            t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
        }
        *reinterpret_cast<float4 *>(partials + (int64_t)blockIdx.x * C + 4 * c4) = t;
    }
}

// Generic C (e.g. 1 value column, 6 action logits): threads over (row group, column), LDS combine.
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd_colsum_scalar(const float *dh, const float *__restrict__ h, int64_t B,
                                                             int C, float slope, float *dz,
                                                             float *__restrict__ partials) {
    __shared__ float s_acc[256];
    const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
    const int64_t r1 = r0 + kRowsPerBlock < B ? r0 + kRowsPerBlock : B;
    for (int cbase = 0; cbase < C; cbase += 256) {
        const int dc = C - cbase < 256 ? C - cbase : 256;
        const int groups = 256 / dc;
        const int c = threadIdx.x % dc, g = threadIdx.x / dc;
        float acc = 0.f;
        if (g < groups) {
#pragma unroll 4
            for (int64_t r = r0 + g; r < r1; r += groups) {
                const int64_t off = r * C + cbase + c;
                float d = dh[off];
                if (ACT != 0) {
                    d = act_grad<ACT>(d, h[off], slope);
                    if (dz) dz[off] = d;
                }
                acc += d;
            }
        }
        s_acc[threadIdx.x] = acc;
        __syncthreads();
        if ((int)threadIdx.x < dc) {
            float t = 0.f;
            for (int k = 0; k < groups; ++k) t += s_acc[k * dc + threadIdx.x];
            partials[(int64_t)blockIdx.x * C + cbase + threadIdx.x] = t;
        }
        __syncthreads();
    }
}

// K11: backward of a thin output layer (K outputs, no activation) and the activation of the hidden
// layer that feeds it, in one pass.  Thread = hidden column i, block = kHeadRows rows:
//   dh[b,i]  = sum_o d_head[b,o] W[o,i]           (the output layer's dX)
//   dz[b,i]  = dh[b,i] * act'(h[b,i])               (hidden activation backward)
//   dW[o,i] += d_head[b,o] h[b,i];  db_h[i] += dz[b,i];  db_o[o] += d_head[b,o]
// W's column and the K accumulators live in registers (KMAX compile-time, K <= KMAX runtime);
// d_head rows are staged in LDS.  Per-block partials are reduced by xpa_colsum_finalize.
constexpr int kHeadRows = 128;

template <int KMAX, int ACT>
__global__ __launch_bounds__(256) void head_backward_kernel(int K, const float *__restrict__ d_head, int64_t ldd,
                                                            const float *__restrict__ h, const float *__restrict__ W,
                                                            int64_t B, int H, float slope, float *__restrict__ dz,
                                                            float *__restrict__ p_dw, float *__restrict__ p_dbh,
                                                            float *__restrict__ p_dbo) {
    __shared__ float s_dh[kHeadRows * KMAX];
    const int64_t r0 = (int64_t)blockIdx.x * kHeadRows;
    const int nr = (int)(B - r0 < kHeadRows ? B - r0 : kHeadRows);
    for (int e = threadIdx.x; e < nr * K; e += 256) {
        const int r = e / K, o = e - r * K;
        s_dh[r * KMAX + o] = d_head[(r0 + r) * ldd + o];
    }
    __syncthreads();
    if ((int)threadIdx.x < K && p_dbo) {  // output-layer bias gradient partial
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s += s_dh[r * KMAX + threadIdx.x];
        p_dbo[(int64_t)blockIdx.x * K + threadIdx.x] = s;
    }
    for (int i = threadIdx.x; i < H; i += 256) {
        float w[KMAX], acc[KMAX];
#pragma unroll
        for (int o = 0; o < KMAX; ++o) {
            w[o] = o < K ? W[(int64_t)o * H + i] : 0.f;
            acc[o] = 0.f;
        }
        float dbh = 0.f;
#pragma unroll 4
        for (int r = 0; r < nr; ++r) {
            const int64_t off = (r0 + r) * H + i;
            const float hv = h[off];
            float d = 0.f;
#pragma unroll
            for (int o = 0; o < KMAX; ++o) {
                if (o < K) {
                    const float g = s_dh[r * KMAX + o];
                    d += g * w[o];
                    acc[o] += g * hv;
                }
            }
            d = act_grad<ACT>(d, hv, slope);
            dz[off] = d;
            dbh += d;
        }
#pragma unroll
        for (int o = 0; o < KMAX; ++o)
            if (o < K) p_dw[((int64_t)blockIdx.x * K + o) * H + i] = acc[o];
        p_dbh[(int64_t)blockIdx.x * H + i] = dbh;
    }
}

// Same computation with 16-B accesses for K <= KMAX <= 8 and hidden % 4 == 0, hidden / 4 <= 256:
// a thread owns 4 consecutive columns of one of (256 / (hidden/4)) row groups, the groups' partial
// accumulators are combined through LDS in a fixed order.
template <int KMAX, int ACT>
__global__ __launch_bounds__(256) void head_backward_vec4_kernel(int K, const float *__restrict__ d_head, int64_t ldd,
                                                                 const float *__restrict__ h,
                                                                 const float *__restrict__ W, int64_t B, int H,
                                                                 float slope, float *__restrict__ dz,
                                                                 float *__restrict__ p_dw, float *__restrict__ p_dbh,
                                                                 float *__restrict__ p_dbo) {
    __shared__ float s_dh[kHeadRows * KMAX];
    __shared__ __attribute__((aligned(16))) float4 s_red[256];
    const int64_t r0 = (int64_t)blockIdx.x * kHeadRows;
    const int nr = (int)(B - r0 < kHeadRows ? B - r0 : kHeadRows);
    for (int e = threadIdx.x; e < nr * K; e += 256) {
        const int r = e / K, o = e - r * K;
        s_dh[r * KMAX + o] = d_head[(r0 + r) * ldd + o];
    }
    __syncthreads();
    if ((int)threadIdx.x < K && p_dbo) {
        float s = 0.f;
        for (int r = 0; r < nr; ++r) s += s_dh[r * KMAX + threadIdx.x];
        p_dbo[(int64_t)blockIdx.x * K + threadIdx.x] = s;
    }
    const int cq = H / 4, groups = 256 / cq;
    const int c4 = threadIdx.x % cq, grp = threadIdx.x / cq;
    float4 w[KMAX], acc[KMAX];
#pragma unroll
    for (int o = 0; o < KMAX; ++o) {
        w[o] = o < K ? *reinterpret_cast<const float4 *>(W + (int64_t)o * H + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 dbh = make_float4(0.f, 0.f, 0.f, 0.f);
    if (grp < groups) {
#pragma unroll 8
        for (int r = grp; r < nr; r += groups) {
            const int64_t off = (r0 + r) * H + 4 * c4;
            const float4 hv = *reinterpret_cast<const float4 *>(h + off);
            float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int o = 0; o < KMAX; ++o) {
                if (o < K) {
                    const float g = s_dh[r * KMAX + o];
                    d.x += g * w[o].x; d.y += g * w[o].y; d.z += g * w[o].z; d.w += g * w[o].w;
                    acc[o].x += g * hv.x; acc[o].y += g * hv.y; acc[o].z += g * hv.z; acc[o].w += g * hv.w;
                }
            }
            d.x = act_grad<ACT>(d.x, hv.x, slope);
            d.y = act_grad<ACT>(d.y, hv.y, slope);
            d.z = act_grad<ACT>(d.z, hv.z, slope);
            d.w = act_grad<ACT>(d.w, hv.w, slope);
            *reinterpret_cast<float4 *>(dz + off) = d;
            dbh.x += d.x; dbh.y += d.y; dbh.z += d.z; dbh.w += d.w;
        }
    }
    // Combine the row groups: one LDS round per accumulator (fixed group order).
    auto combine = [&](float4 v, float *dst) {
        s_red[threadIdx.x] = v;
        __syncthreads();
        if (grp == 0) {
            float4 t = s_red[c4];
            for (int g2 = 1; g2 < groups; ++g2) {
                const float4 a = s_red[g2 * cq + c4];
                t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
            }
            *reinterpret_cast<float4 *>(dst + 4 * c4) = t;
        }
        __syncthreads();
    };
#pragma unroll
    for (int o = 0; o < KMAX; ++o)
        if (o < K) combine(acc[o], p_dw + ((int64_t)blockIdx.x * K + o) * H);
    combine(dbh, p_dbh + (int64_t)blockIdx.x * H);
}

// Column sums of per-block partials [G, C] -> out [C]: a block owns 64 columns (coalesced 256-B row
// reads) x 16 row groups (thread (g, c) sums rows g, g + 16, ... in order, f64); the groups are combined
// through LDS in a fixed order -> deterministic, and identical for the single and the batched entry.
constexpr int kColTile = 64;
constexpr int kColGroups = 16;

// sq != nullptr: also the tile's sum of squared outputs (f64, wave 0) into *sq — the gradient-norm
// partial the clip + Adam step reads (xpa_clip_adam_step_partials), in place of a separate norm pass.
// Output map (r05; tm_inner = 0: out[c]): column c = r tm_inner + i of the partials goes to out[i tm_ld + r] when
// r < tm_valid and is dropped otherwise — a transposed, row-trimmed store (K41V's x^T dz slices of the C4 trunk layer,
// [384 padded inputs][256] -> dW [256][376])
__device__ __forceinline__ bool colsum_put(float *__restrict__ out, int c, float o, int tm_inner, int tm_valid,
                                           int64_t tm_ld) {
    if (tm_inner == 0) {
        out[c] = o;
        return true;
    }
    const int r = c / tm_inner, i = c - r * tm_inner;
    if (r >= tm_valid) return false;
    out[(int64_t)i * tm_ld + r] = o;
    return true;
}

__device__ __forceinline__ void colsum_tile(const float *__restrict__ part, int64_t G, int C, int c0,
                                            float *__restrict__ out, double (*s_red)[kColTile],
                                            double *__restrict__ sq = nullptr, int tm_inner = 0, int tm_valid = 0,
                                            int64_t tm_ld = 0) {
    const int lane = threadIdx.x & (kColTile - 1), grp = threadIdx.x / kColTile;
    const int c = c0 + lane;
    double s = 0.0;
    if (c < C) {
        int64_t k = grp;
        for (; k + 15 * kColGroups < G; k += 16 * kColGroups) {  // 16 independent loads in flight (G = 512: 2 rounds)
            float a[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u] = part[(k + u * kColGroups) * C + c];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += (double)a[u];
        }
        for (; k + 3 * kColGroups < G; k += 4 * kColGroups) {  // 4 independent loads in flight
            const float a0 = part[k * C + c], a1 = part[(k + kColGroups) * C + c];
            const float a2 = part[(k + 2 * kColGroups) * C + c], a3 = part[(k + 3 * kColGroups) * C + c];
            s += (double)a0;
            s += (double)a1;
            s += (double)a2;
            s += (double)a3;
        }
        for (; k < G; k += kColGroups) s += (double)part[k * C + c];
    }
    s_red[grp][lane] = s;
    __syncthreads();
    if (grp == 0) {
        float o = 0.f;
        if (c < C) {
            double t = s_red[0][lane];
            for (int g = 1; g < kColGroups; ++g) t += s_red[g][lane];
            o = (float)t;
            if (!colsum_put(out, c, o, tm_inner, tm_valid, tm_ld)) o = 0.f;
        }
        if (sq) {  // grp 0 is wave 0 (kColTile == 64)
            const double q = xpa_wave_sum((double)o * (double)o);
            if (lane == 0) xpa_store_agent(sq, q);
        }
    }
}

__global__ __launch_bounds__(kColTile * kColGroups) void colsum_finalize_kernel(const float *__restrict__ partials,
                                                                               int64_t G, int C,
                                                                               float *__restrict__ out) {
    __shared__ double s_red[kColGroups][kColTile];
    colsum_tile(partials, G, C, (int)blockIdx.x * kColTile, out, s_red);
}

constexpr int kMaxSegs = 16;
// the batched finalize's ticket buffer (ABI 4): int32 [kColTicketStride (1 + kColTicketGroups)] = XPA_COLSUM_TICKET_INTS
constexpr unsigned kColTicketStride = 64, kColTicketGroups = 63;
static_assert(kColTicketStride * (1 + kColTicketGroups) == XPA_COLSUM_TICKET_INTS, "ticket buffer size (ABI 4)");
// Segments with few partial rows (G <= kWideMaxG, e.g. the split-K slices of a weight gradient: G = 8,
// C = 131 072) use 1024-column tiles, one column per thread summed over G in order; the others 64-column
// tiles with 16 row groups (colsum_tile).
constexpr int kWideTile = kColTile * kColGroups;
constexpr int kWideMaxG = 32;

// Segments with 32 < G <= 256 (K41's 64 weight-gradient slices over C = 131 072): 512-column tiles, 4 row groups of
// 256 threads (rows grp, grp + 4, ...; 2 columns c, c + 256 per thread, 16 loads in flight each), the groups added in
// order in f64 — r04: the 64-column tiles of colsum_tile took 32 us for K41's 32 MiB; 256-column tiles (one column per
// thread) 20 us, their 512 blocks + the other segments' spilling into a second round of blocks (2 per CU).
constexpr int kMidTile = 512;
constexpr int kMidMaxG = 256;
__host__ __device__ inline int64_t seg_tiles(int64_t G, int64_t C) {
    return G <= kWideMaxG ? (C + kWideTile - 1) / kWideTile
                          : G <= kMidMaxG ? (C + kMidTile - 1) / kMidTile : (C + kColTile - 1) / kColTile;
}

struct ColsumBatch {
    const float *part[kMaxSegs];
    float *out[kMaxSegs];
    int64_t G[kMaxSegs];
    int C[kMaxSegs];
    int tile0[kMaxSegs + 1];  // first column tile of each segment
    int tm_inner[kMaxSegs], tm_valid[kMaxSegs];   // output maps (colsum_put; 0 = identity)
    int64_t tm_ld[kMaxSegs];
    int n;
    // nullable: clip-norm partials.  sq[0] = a share written beforehand (d logstd, loss finalize),
    // sq[1 + tile] = each tile's sum of squared outputs, and the last block to finish (ticket) writes
    // the fixed-order total of sq[0 .. tiles] into sq[1 + tiles] and resets the ticket.
    double *sq;
    unsigned int *ticket;
    // has_loss: the LAST block runs the loss finalize (xpa_loss_finalize_body) instead of a column tile,
    // writing its d logstd share into sq[0] before taking its ticket
    int has_loss;
    XpaLossFinalizeArgs loss;
};

// One column tile of a batched finalize (sq: this tile's squared-sum slot or nullptr).
__device__ __forceinline__ void colsum_batch_tile(const ColsumBatch &b, int tile, double *sq,
                                                  double (*s_red)[kColTile]) {
    int sg = 0;
    while (tile >= b.tile0[sg + 1]) ++sg;
    if (b.G[sg] <= kWideMaxG) {
        const int64_t G = b.G[sg];
        const int C = b.C[sg];
        const int c = (tile - b.tile0[sg]) * kWideTile + (int)threadIdx.x;
        const float *part = b.part[sg];
        double acc = 0.0;
        float o = 0.f;
        if (c < C) {
            int64_t k = 0;
            for (; k + 8 <= G; k += 8) {  // 8 loads in flight, added in row order
                float a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) a[u] = part[(k + u) * C + c];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += (double)a[u];
            }
            for (; k < G; ++k) acc += (double)part[k * C + c];
            o = (float)acc;
            if (!colsum_put(b.out[sg], c, o, b.tm_inner[sg], b.tm_valid[sg], b.tm_ld[sg])) o = 0.f;
        }
        if (sq) {
            const double q = xpa_wave_sum((double)o * (double)o);
            if ((threadIdx.x & 63) == 0) s_red[0][threadIdx.x >> 6] = q;
            __syncthreads();
            if (threadIdx.x == 0) {
                double t = 0.0;
                for (int w = 0; w < kWideTile / 64; ++w) t += s_red[0][w];
                xpa_store_agent(sq, t);
            }
        }
    } else if (b.G[sg] <= kMidMaxG) {
        static_assert(kColGroups * kColTile == 4 * 256, "the mid path reuses s_red as [4][256]");
        auto s4 = reinterpret_cast<double(*)[256]>(s_red);
        const int64_t G = b.G[sg];
        const int C = b.C[sg];
        const int grp = threadIdx.x >> 8, lc = threadIdx.x & 255;
        const int c0 = (tile - b.tile0[sg]) * kMidTile + lc;
        const float *part = b.part[sg];
        double acc[2] = {0.0, 0.0};
        {
            int64_t k = grp;
            for (; k + 15 * 4 < G; k += 16 * 4) {  // 2 x 16 loads in flight, each column added in row order
                float a[2][16];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = min(c0 + 256 * h, C - 1);
#pragma unroll
                    for (int u = 0; u < 16; ++u) a[h][u] = part[(k + 4 * u) * C + c];
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int u = 0; u < 16; ++u) acc[h] += (double)a[h][u];
            }
            for (; k < G; k += 4) {
#pragma unroll
                for (int h = 0; h < 2; ++h) acc[h] += (double)part[k * C + min(c0 + 256 * h, C - 1)];
            }
        }
        float o[2] = {0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 2; ++h) {   // the 4 groups of column set h, added in order
            if (h) __syncthreads();       // set 0's s4 reads done
            s4[grp][lc] = acc[h];
            __syncthreads();
            const int c = c0 + 256 * h;
            if (grp == 0 && c < C) {
                o[h] = (float)(((s4[0][lc] + s4[1][lc]) + s4[2][lc]) + s4[3][lc]);
                if (!colsum_put(b.out[sg], c, o[h], b.tm_inner[sg], b.tm_valid[sg], b.tm_ld[sg])) o[h] = 0.f;
            }
        }
        if (sq) {
            __syncthreads();   // s4 read by group 0: its slots reused for the wave sums
            const double q = xpa_wave_sum((double)o[0] * (double)o[0] + (double)o[1] * (double)o[1]);
            if ((threadIdx.x & 63) == 0 && grp == 0) s4[1][threadIdx.x >> 6] = q;
            __syncthreads();
            if (threadIdx.x == 0) xpa_store_agent(sq, ((s4[1][0] + s4[1][1]) + s4[1][2]) + s4[1][3]);
        }
    } else {
        colsum_tile(b.part[sg], b.G[sg], b.C[sg], (tile - b.tile0[sg]) * kColTile, b.out[sg], s_red, sq,
                    b.tm_inner[sg], b.tm_valid[sg], b.tm_ld[sg]);
    }
}

__global__ __launch_bounds__(kColTile * kColGroups) void colsum_finalize_batch_kernel(ColsumBatch b) {
    __shared__ double s_red[kColGroups][kColTile];
    __shared__ bool s_last;
    const int tile = blockIdx.x;
    if (b.has_loss && tile == (int)gridDim.x - 1) {  // the loss finalize block (its share into sq[0])
        __shared__ double s_tot[kXpaLossPartBase];
        __shared__ float s_dls[kXpaLossMaxAct];
        xpa_loss_finalize_body(b.loss, b.sq, s_tot, s_dls);
    } else {
        colsum_batch_tile(b, tile, b.sq ? b.sq + 1 + tile : nullptr, s_red);
    }
    if (!b.sq) return;
    xpa_drain();  // this block's partial (sc1 store) complete before its ticket
    __syncthreads();
    // r06 (ABI 4): two ticket levels on separate 256-B lines — the blocks of group g (kColTicketGroups groups of
    // contiguous blocks) count on ticket[kColTicketStride (1 + g)], each group's last block on ticket[0]: one counter for
    // all ~300 tiles of a C2 update serialised their atomics on one line (K14F measured ~19 ns per atomic per line)
    if (threadIdx.x == 0) {
        const unsigned nb = gridDim.x;
        const unsigned gs = (nb + kColTicketGroups - 1) / kColTicketGroups, ng = (nb + gs - 1) / gs;
        const unsigned g = blockIdx.x / gs, gn = min(gs, nb - g * gs);
        unsigned *gt = b.ticket + kColTicketStride * (1 + g);
        bool last = xpa_ticket(gt) == gn - 1;
        if (last) {
            *gt = 0u;   // every block of the group has taken its ticket
            last = xpa_ticket(b.ticket) == ng - 1;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    const int n = (int)gridDim.x + (b.has_loss ? 0 : 1);  // sq[0 .. tiles]
    // thread t sums a contiguous run of the partials in order, then the runs in thread order (fixed)
    const int per = (n + kWideTile - 1) / kWideTile;
    double acc = 0.0;
    for (int i = threadIdx.x * per; i < n && i < ((int)threadIdx.x + 1) * per; ++i) acc += xpa_load_agent(b.sq + i);
    __shared__ double s_all[kWideTile];
    s_all[threadIdx.x] = acc;
    __syncthreads();
    for (int off = kWideTile / 2; off > 0; off >>= 1) {  // fixed-shape tree: deterministic
        if ((int)threadIdx.x < off) s_all[threadIdx.x] += s_all[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        b.sq[n] = s_all[0];
        *b.ticket = 0u;
    }
}

}  // namespace

XPA_API int64_t xpa_act_bwd_num_partials(int64_t rows) { return (rows + kRowsPerBlock - 1) / kRowsPerBlock; }

XPA_API int xpa_act_bwd_colsum(int act, const float *dh, const float *h, int64_t rows, int64_t cols, float slope,
                               float *dz, float *partials, xpa_stream_t stream) {
    if (rows <= 0 || cols <= 0 || cols > (1 << 20) || !dh || !partials || act < 0 || act > 2)
        return (int)hipErrorInvalidValue;
    if (act != 0 && !h) return (int)hipErrorInvalidValue;
    const int64_t G = xpa_act_bwd_num_partials(rows);
    const int C = (int)cols;
    hipStream_t s = (hipStream_t)stream;
    const bool vec = (C % 4 == 0) && (C / 4 <= 256) &&
                     (((uintptr_t)dh | (uintptr_t)(h ? h : dh) | (uintptr_t)(dz ? dz : dh) | (uintptr_t)partials) % 16 == 0);
    if (vec) {
        const int cq = C / 4;
        const int groups = 256 / cq;
        const size_t lds = (size_t)groups * cq * sizeof(float4);
#define XPA_ACT_LAUNCH(A_)                                                                                        \
    hipLaunchKernelGGL((act_bwd_colsum_vec4<A_>), dim3((unsigned)G), dim3(256), lds, s, dh, h, rows, C, slope, dz, \
                       partials)
        if (act == 0) XPA_ACT_LAUNCH(0);
        else if (act == 1) XPA_ACT_LAUNCH(1);
        else XPA_ACT_LAUNCH(2);
#undef XPA_ACT_LAUNCH
    } else {
#define XPA_ACT_LAUNCH(A_)                                                                                          \
    hipLaunchKernelGGL((act_bwd_colsum_scalar<A_>), dim3((unsigned)G), dim3(256), 0, s, dh, h, rows, C, slope, dz, \
                       partials)
        if (act == 0) XPA_ACT_LAUNCH(0);
        else if (act == 1) XPA_ACT_LAUNCH(1);
        else XPA_ACT_LAUNCH(2);
#undef XPA_ACT_LAUNCH
    }
    return xpa_launch_status();
}

XPA_API int64_t xpa_head_bwd_num_partials(int64_t rows) { return (rows + kHeadRows - 1) / kHeadRows; }

XPA_API int xpa_head_backward(int act, int64_t k, const float *d_head, int64_t ldd, const float *h, const float *w,
                              int64_t rows, int64_t hidden, float slope, float *dz, float *partial_dw,
                              float *partial_db_hidden, float *partial_db_out, xpa_stream_t stream) {
    if (rows <= 0 || hidden <= 0 || k <= 0 || k > 32 || ldd < k || act < 0 || act > 2 || !d_head || !h || !w ||
        !dz || !partial_dw || !partial_db_hidden)
        return (int)hipErrorInvalidValue;
    const unsigned G = (unsigned)xpa_head_bwd_num_partials(rows);
    hipStream_t s = (hipStream_t)stream;
    const int K = (int)k, H = (int)hidden;
#define XPA_HEAD_LAUNCH(KM_, A_)                                                                                    \
    hipLaunchKernelGGL((head_backward_kernel<KM_, A_>), dim3(G), dim3(256), 0, s, K, d_head, ldd, h, w, rows, H,   \
                       slope, dz, partial_dw, partial_db_hidden, partial_db_out)
#define XPA_HEAD_ACT(KM_)                 \
    do {                                  \
        if (act == 0) XPA_HEAD_LAUNCH(KM_, 0); \
        else if (act == 1) XPA_HEAD_LAUNCH(KM_, 1); \
        else XPA_HEAD_LAUNCH(KM_, 2);     \
    } while (0)
    const bool vec = (H % 4 == 0) && (H / 4 <= 256) && K <= 8 &&
                     (((uintptr_t)h | (uintptr_t)w | (uintptr_t)dz | (uintptr_t)partial_dw | (uintptr_t)partial_db_hidden) %
                      16 == 0);
    if (vec) {
#undef XPA_HEAD_LAUNCH
#define XPA_HEAD_LAUNCH(KM_, A_)                                                                                     \
    hipLaunchKernelGGL((head_backward_vec4_kernel<KM_, A_>), dim3(G), dim3(256), 0, s, K, d_head, ldd, h, w, rows, H, \
                       slope, dz, partial_dw, partial_db_hidden, partial_db_out)
        if (K == 1) XPA_HEAD_ACT(1);
        else if (K <= 2) XPA_HEAD_ACT(2);
        else XPA_HEAD_ACT(8);
    } else {
#undef XPA_HEAD_LAUNCH
#define XPA_HEAD_LAUNCH(KM_, A_)                                                                                    \
    hipLaunchKernelGGL((head_backward_kernel<KM_, A_>), dim3(G), dim3(256), 0, s, K, d_head, ldd, h, w, rows, H,   \
                       slope, dz, partial_dw, partial_db_hidden, partial_db_out)
        if (K == 1) XPA_HEAD_ACT(1);
        else if (K <= 8) XPA_HEAD_ACT(8);
        else XPA_HEAD_ACT(32);
    }
#undef XPA_HEAD_ACT
#undef XPA_HEAD_LAUNCH
    return xpa_launch_status();
}

XPA_API int xpa_colsum_finalize(const float *partials, int64_t n_partials, int64_t cols, float *out,
                                xpa_stream_t stream) {
    if (n_partials <= 0 || cols <= 0 || !partials || !out) return (int)hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((cols + kColTile - 1) / kColTile);
    hipLaunchKernelGGL(colsum_finalize_kernel, dim3(blocks), dim3(kColTile * kColGroups), 0, (hipStream_t)stream,
                       partials, n_partials, (int)cols, out);
    return xpa_launch_status();
}

XPA_API int64_t xpa_colsum_batch_tiles(int n_segs, const int64_t *n_partials, const int64_t *cols) {
    int64_t tiles = 0;
    for (int i = 0; i < n_segs; ++i) tiles += seg_tiles(n_partials[i], cols[i]);
    return tiles;
}

namespace {
int colsum_batch_launch(int n_segs, const float *const *partials, const int64_t *n_partials, const int64_t *cols,
                        float *const *outs, double *sq, int32_t *ticket, const XpaLossFinalizeArgs *loss,
                        xpa_stream_t stream, const int64_t *tmap = nullptr) {
    if (n_segs <= 0 || n_segs > kMaxSegs || !partials || !n_partials || !cols || !outs) return (int)hipErrorInvalidValue;
    if (sq && !ticket) return (int)hipErrorInvalidValue;
    ColsumBatch b{};
    b.sq = sq;
    b.ticket = (unsigned int *)ticket;
    if (loss) {
        b.has_loss = 1;
        b.loss = *loss;
    }
    b.n = n_segs;
    int64_t tiles = 0;
    for (int i = 0; i < n_segs; ++i) {
        if (!partials[i] || !outs[i] || n_partials[i] <= 0 || cols[i] <= 0 || cols[i] > (1 << 24))
            return (int)hipErrorInvalidValue;
        b.part[i] = partials[i];
        b.out[i] = outs[i];
        b.G[i] = n_partials[i];
        b.C[i] = (int)cols[i];
        if (tmap && tmap[3 * i] != 0) {   // (inner, valid, ld): C = rows x inner, valid <= rows, ld >= valid
            const int64_t in = tmap[3 * i], va = tmap[3 * i + 1], ld = tmap[3 * i + 2];
            if (in < 1 || cols[i] % in != 0 || va < 1 || va > cols[i] / in || ld < va) return (int)hipErrorInvalidValue;
            b.tm_inner[i] = (int)in;
            b.tm_valid[i] = (int)va;
            b.tm_ld[i] = ld;
        }
        b.tile0[i] = (int)tiles;
        tiles += seg_tiles(n_partials[i], cols[i]);
    }
    b.tile0[n_segs] = (int)tiles;
    hipLaunchKernelGGL(colsum_finalize_batch_kernel, dim3((unsigned)(tiles + (loss ? 1 : 0))),
                       dim3(kColTile * kColGroups), 0, (hipStream_t)stream, b);
    return xpa_launch_status();
}
}  // namespace

XPA_API int xpa_colsum_finalize_batch_sq(int n_segs, const float *const *partials, const int64_t *n_partials,
                                         const int64_t *cols, float *const *outs, double *sq, int32_t *ticket,
                                         xpa_stream_t stream) {
    return colsum_batch_launch(n_segs, partials, n_partials, cols, outs, sq, ticket, nullptr, stream);
}

XPA_API int xpa_colsum_finalize_batch_sq_loss(int n_segs, const float *const *partials, const int64_t *n_partials,
                                              const int64_t *cols, float *const *outs, double *sq, int32_t *ticket,
                                              int algo, int dist, int64_t batch, int64_t act_dim,
                                              const float *loss_partials, int64_t n_loss_partials, float vf_coef,
                                              float ent_coef, float *scalars, float *d_logstd,
                                              xpa_stream_t stream) {
    if (!sq || !ticket || batch <= 0 || act_dim <= 0 || act_dim > kXpaLossMaxAct || n_loss_partials <= 0 ||
        !loss_partials || !scalars || (dist == XPA_DIST_GAUSSIAN && !d_logstd))
        return (int)hipErrorInvalidValue;
    const XpaLossFinalizeArgs loss{algo, dist, batch, (int)act_dim, loss_partials, n_loss_partials,
                                   (int)xpa_loss_partial_width(act_dim), vf_coef, ent_coef, scalars, d_logstd};
    return colsum_batch_launch(n_segs, partials, n_partials, cols, outs, sq, ticket, &loss, stream);
}

// r05: the batched finalizes with per-segment output maps tmap [n_segs][3] = (inner, valid, ld) (inner 0: identity;
// else column r inner + i -> out[i ld + r] for r < valid, dropped otherwise); sq / ticket nullable as a pair; with
// loss_partials the loss finalize block as in xpa_colsum_finalize_batch_sq_loss (algo .. d_logstd ignored otherwise)
XPA_API int xpa_colsum_finalize_batch_map(int n_segs, const float *const *partials, const int64_t *n_partials,
                                          const int64_t *cols, float *const *outs, const int64_t *tmap, double *sq,
                                          int32_t *ticket, int algo, int dist, int64_t batch, int64_t act_dim,
                                          const float *loss_partials, int64_t n_loss_partials, float vf_coef,
                                          float ent_coef, float *scalars, float *d_logstd, xpa_stream_t stream) {
    if (!tmap) return (int)hipErrorInvalidValue;
    if (!loss_partials) return colsum_batch_launch(n_segs, partials, n_partials, cols, outs, sq, ticket, nullptr, stream,
                                                   tmap);
    if (!sq || !ticket || batch <= 0 || act_dim <= 0 || act_dim > kXpaLossMaxAct || n_loss_partials <= 0 || !scalars ||
        (dist == XPA_DIST_GAUSSIAN && !d_logstd))
        return (int)hipErrorInvalidValue;
    const XpaLossFinalizeArgs loss{algo, dist, batch, (int)act_dim, loss_partials, n_loss_partials,
                                   (int)xpa_loss_partial_width(act_dim), vf_coef, ent_coef, scalars, d_logstd};
    return colsum_batch_launch(n_segs, partials, n_partials, cols, outs, sq, ticket, &loss, stream, tmap);
}

XPA_API int xpa_colsum_finalize_batch(int n_segs, const float *const *partials, const int64_t *n_partials,
                                      const int64_t *cols, float *const *outs, xpa_stream_t stream) {
    return xpa_colsum_finalize_batch_sq(n_segs, partials, n_partials, cols, outs, nullptr, nullptr, stream);
}
