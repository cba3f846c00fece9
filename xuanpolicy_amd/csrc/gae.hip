// K1 — GAE / discounted-return reverse scan over a [n_envs, horizon] rollout buffer (gfx950).
//
// Replaces DummyOnPolicyBuffer.finish_path (reference xuance/common/memory_tools.py:206-229) as
// called by the agent at every path closure (ppoclip_agent.py:69-101): instead of one Python loop per
// path, the closures are recorded as per-(env, step) flags and the whole buffer is scanned once.
//
// Recurrence (per element t of a row; "closed" = a path ends at t with bootstrap boot[t]):
//   nv_t = closed_t ? boot_t : v_{t+1}
//   GAE:     A_t = b_t + a_t A_{t+1},  b_t = r_t + g(1-d_t) nv_t - v_t,  a_t = closed_t ? 0 : g l (1-d_t)
//            R_t = A_t + v_t
//   returns: R_t = b_t + a_t R_{t+1},  b_t = r_t + (closed_t ? g boot_t : 0), a_t = closed_t ? 0 : g
//            A_t = r_t + g nv_t - v_t          (no done mask: discount_cumsum branch, memory_tools.py:222-225)
// A_t = b_t + a_t A_{t+1} is an affine map; maps compose associatively,
//   (a1, b1) o (a2, b2) = (a1 a2, b1 + a1 b2),
// so a row is a reverse inclusive scan.  Mapping on CDNA4:
//   * a row of T steps is a segment of L = min(64, pow2 >= T/VEC) lanes of one wave64; a wave holds
//     64/L rows (T = 128: two rows per wave, 32 lanes each);
//   * each lane owns VEC = 4 consecutive steps: every load/store is a 16-B float4 (1 KiB per wave
//     instruction, fully coalesced over the row-major [N, T] layout), flags as one u8x4;
//   * a lane first composes its 4 maps in registers, then the segment runs a log2(L)-step
//     reverse scan with cross-lane shuffles (ds_bpermute, no LDS footprint), then each lane expands
//     its 4 outputs; rows longer than 64*VEC loop over chunks from the end with a register carry;
//   * the boot value is read only where closed (sparse); positions after the last closure of a row
//     (an open path) are not written, exactly like the reference.
//   * boot is streamed densely alongside r, v, d (vector path): reading it only where closed made a
//     dependent second memory round trip in every wave (each row closes at its last step at rollout
//     end) — 0.9-2.1 us of a 5-7 us launch at 4096 x 128 (tools/gae_floor.hip, r01).
// Algorithmic bytes: 20 B per (env, step) (r, v, d read; adv, ret written); this
// kernel moves 25 B (+1 B closure flag, +4 B boot).
#include <stdlib.h>

#include <hip/hip_ext.h>

#include "xpa_common.h"

namespace {

// NT = 1: non-temporal (streaming) 16-B loads/stores — every byte is touched exactly once.
typedef float f4v __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ float4 ld4(const float *p) {
    if (NT) {
        const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
        return make_float4(x[0], x[1], x[2], x[3]);
    }
    return *reinterpret_cast<const float4 *>(p);
}

template <int NT>
__device__ __forceinline__ void st4(float *p, float4 v) {
    if (NT) {
        __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v *>(p));
    } else {
        *reinterpret_cast<float4 *>(p) = v;
    }
}

// COMPACT = 1 (the fused agent's rollout with deferred truncation bootstraps, non-Atari): no closure
// flags and no dense boot stream.  A row closes at its terminals (d != 0), at its one mid-buffer
// truncation slot_t[row] (K8 records at most one per rollout) and at its last step; the bootstraps are
// the critic values vboot[row] (truncation slot) and vboot[n_rows + row] (last step, 0 when terminal),
// loaded once per row next to the r/v/d streams.  The kernel writes those two bootstraps into `boot`
// (the buffer's state is that of xpa_rollout_bootstrap_fixup + xpa_gae_scan) and resets slot_t.
// Bytes: exactly the algorithmic 20 B per (env, step) + 12 B per env (+8 B sparse boot writes).
template <int VEC, int NT, int COMPACT = 0>
__global__ __launch_bounds__(256) void gae_scan_kernel(const float *__restrict__ rew, const float *__restrict__ val,
                                                       const float *__restrict__ term,
                                                       const uint8_t *__restrict__ closed,
                                                       const float *__restrict__ boot, int64_t n_rows, int T,
                                                       int seg_log2, float gamma, float gl, int use_gae,
                                                       float *__restrict__ adv, float *__restrict__ ret,
                                                       int *__restrict__ slot_t = nullptr,
                                                       const float *__restrict__ vboot = nullptr,
                                                       float *__restrict__ boot_out = nullptr) {
    const int L = 1 << seg_log2;
    const int lane = threadIdx.x & 63;
    const int sl = lane & (L - 1);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t row = wave * (64 >> seg_log2) + (lane >> seg_log2);
    const bool row_ok = row < n_rows;
    const int64_t base = row_ok ? row * (int64_t)T : 0;
    const int C = L * VEC;
    const int nchunks = (T + C - 1) / C;

    int st = -1;
    float vs = 0.f, vl = 0.f;
    if (COMPACT && row_ok) {
        st = slot_t[row];
        vs = vboot[row];
        vl = vboot[n_rows + row];
    }

    float carry = 0.f;   // A (or R) at the first element of the later chunk
    float carry_v = 0.f; // v at that element
    int carry_any = 0;   // a closure exists at or after the later chunk's first element
    bool has_last = false;  // compact form: this lane owns step T - 1 of its row
    float last_boot = 0.f;

    for (int c = nchunks - 1; c >= 0; --c) {
        const int t0 = c * C + sl * VEC;
        float r[VEC], v[VEC], d[VEC], bt[VEC];
        int cl[VEC];
        const bool full = row_ok && (t0 + VEC <= T);
        if (COMPACT && VEC == 4 && full) {
            const float4 r4 = ld4<NT>(rew + base + t0);
            const float4 v4 = ld4<NT>(val + base + t0);
            const float4 d4 = ld4<NT>(term + base + t0);
            r[0] = r4.x; r[1] = r4.y; r[2] = r4.z; r[3] = r4.w;
            v[0] = v4.x; v[1] = v4.y; v[2] = v4.z; v[3] = v4.w;
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z; d[3] = d4.w;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const int t = t0 + e;
                const bool lt = (t == T - 1);
                cl[e] = lt || d[e] != 0.f || t == st;
                bt[e] = lt ? (d[e] != 0.f ? 0.f : vl) : (t == st ? vs : 0.f);
                if (lt) {
                    has_last = true;
                    last_boot = bt[e];
                }
            }
        } else if (COMPACT) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const int t = t0 + e;
                const bool ok = row_ok && t < T;
                r[e] = ok ? rew[base + t] : 0.f;
                v[e] = ok ? val[base + t] : 0.f;
                d[e] = ok ? term[base + t] : 0.f;
                const bool lt = (t == T - 1);
                cl[e] = ok && (lt || d[e] != 0.f || t == st);
                bt[e] = lt ? (d[e] != 0.f ? 0.f : vl) : (t == st ? vs : 0.f);
                if (ok && lt) {
                    has_last = true;
                    last_boot = bt[e];
                }
            }
        } else if (VEC == 4 && full) {
            const float4 r4 = ld4<NT>(rew + base + t0);
            const float4 v4 = ld4<NT>(val + base + t0);
            const float4 d4 = ld4<NT>(term + base + t0);
            const uint32_t c4 = *reinterpret_cast<const uint32_t *>(closed + base + t0);  // one dword, 4 flags
            // boot is read densely with the other streams: +4 B per step, but no dependent second
            // round trip after the flags land (every row closes at its last step at rollout end).
            const float4 q4 = ld4<NT>(boot + base + t0);
            bt[0] = q4.x; bt[1] = q4.y; bt[2] = q4.z; bt[3] = q4.w;
            r[0] = r4.x; r[1] = r4.y; r[2] = r4.z; r[3] = r4.w;
            v[0] = v4.x; v[1] = v4.y; v[2] = v4.z; v[3] = v4.w;
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z; d[3] = d4.w;
            cl[0] = c4 & 0xff; cl[1] = (c4 >> 8) & 0xff; cl[2] = (c4 >> 16) & 0xff; cl[3] = c4 >> 24;
        } else {
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const int t = t0 + e;
                const bool ok = row_ok && t < T;
                r[e] = ok ? rew[base + t] : 0.f;
                v[e] = ok ? val[base + t] : 0.f;
                d[e] = ok ? term[base + t] : 0.f;
                cl[e] = ok ? (int)closed[base + t] : 0;
                bt[e] = cl[e] ? boot[base + t] : 0.f;
            }
        }
        // v_{t+1} of this lane's last element: the next lane's first v, or the later chunk's.
        float vn_lane = __shfl_down(v[0], 1, L);
        if (sl == L - 1) vn_lane = carry_v;

        float a[VEC], b[VEC], adv_direct[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            const int t = t0 + e;
            const bool ok = row_ok && t < T;
            const float vnext = (e < VEC - 1) ? v[e + 1] : vn_lane;
            const float nv = cl[e] ? bt[e] : vnext;
            const float nd = 1.0f - d[e];
            if (use_gae) {
                b[e] = r[e] + gamma * nd * nv - v[e];
                a[e] = cl[e] ? 0.f : gl * nd;
            } else {
                b[e] = r[e] + (cl[e] ? gamma * bt[e] : 0.f);
                a[e] = cl[e] ? 0.f : gamma;
                adv_direct[e] = r[e] + gamma * nv - v[e];
            }
            if (!ok) { a[e] = 1.f; b[e] = 0.f; }
        }
        // Lane-local composition (last element first).
        float LA = 1.f, LB = 0.f;
        int lany = 0;
#pragma unroll
        for (int e = VEC - 1; e >= 0; --e) {
            LB = b[e] + a[e] * LB;
            LA = a[e] * LA;
            lany |= cl[e];
        }
        // Segmented reverse inclusive scan across the L lanes of this row.
        for (int o = 1; o < L; o <<= 1) {
            const float oA = __shfl_down(LA, o, L);
            const float oB = __shfl_down(LB, o, L);
            const int oany = __shfl_down(lany, o, L);
            if (sl + o < L) {
                LB = LB + LA * oB;
                LA = LA * oA;
                lany |= oany;
            }
        }
        const float first = LB + LA * carry;
        const int any_first = lany | carry_any;
        float nxt = __shfl_down(first, 1, L);
        int nany = __shfl_down(any_first, 1, L);
        if (sl == L - 1) {
            nxt = carry;
            nany = carry_any;
        }
        float oa[VEC], orr[VEC];
        int wr[VEC];
#pragma unroll
        for (int e = VEC - 1; e >= 0; --e) {
            const float x = b[e] + a[e] * nxt;
            const int anyc = cl[e] | nany;
            if (use_gae) {
                oa[e] = x;
                orr[e] = x + v[e];
            } else {
                oa[e] = adv_direct[e];
                orr[e] = x;
            }
            wr[e] = anyc && row_ok && (t0 + e < T);
            nxt = x;
            nany = anyc;
        }
        if (VEC == 4 && full && wr[0] && wr[1] && wr[2] && wr[3]) {
            st4<NT>(adv + base + t0, make_float4(oa[0], oa[1], oa[2], oa[3]));
            st4<NT>(ret + base + t0, make_float4(orr[0], orr[1], orr[2], orr[3]));
        } else {
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                if (wr[e]) {
                    adv[base + t0 + e] = oa[e];
                    ret[base + t0 + e] = orr[e];
                }
            }
        }
        carry = __shfl(first, 0, L);
        carry_v = __shfl(v[0], 0, L);
        carry_any = __shfl(any_first, 0, L);
    }
    if (COMPACT && has_last) boot_out[base + T - 1] = last_boot;  // from registers (see gae_dpp_kernel)
    if (COMPACT && row_ok && sl == 0) {  // the fixup's writes: the two bootstraps, slot reset
        if (st >= 0 && st < T - 1) boot_out[base + st] = vs;
        if (st >= 0) slot_t[row] = -1;
    }
}


// ---- DPP form (T > 32, 16-B aligned, T % 4 == 0: every rollout buffer) --------------------------------
// The same affine scan with the lane order reversed inside a row segment: lane sl owns the 4 steps
// starting at c*C + (L-1-sl)*4, so the reverse-in-time scan is a forward scan in lane order and runs
// on DPP (row_shr:1/2/4/8, row_bcast:15/31 — ALU-latency lane moves) instead of ds_bpermute round
// trips; the closure "any later" flags come from one ballot, the neighbour values from wave_shr:1.
// (The ds_bpermute form made the 4096 x 128 launch 1.7 us slower than a copy of its bytes, r01 probe
// tools/gae_modes.hip.)
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_mov(float old, float src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                 __builtin_bit_cast(int, src), CTRL, ROW_MASK, 0xf,
                                                                 false));
}
constexpr int kDppRowShr = 0x110, kDppWaveShr1 = 0x138, kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;

template <int O, int CTRL, int ROW_MASK>
__device__ __forceinline__ void dpp_combine(float &LA, float &LB) {
    const float oA = dpp_mov<CTRL, ROW_MASK>(1.f, LA);  // disabled / out-of-row lanes: the identity map
    const float oB = dpp_mov<CTRL, ROW_MASK>(0.f, LB);
    LB = LB + LA * oB;
    LA = LA * oA;
}

// xor-butterfly partner inside a 32-lane group without an LDS round trip (ds_swizzle bitmask mode:
// src lane = ((lane & 0x1f) | 0) ^ X)
template <int X>
__device__ __forceinline__ float swz_xor(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x1f | (X << 10)));
}

// Value-fused form (VACT >= 0, with COMPACT): the deferred bootstraps' critic values are formed here from the
// critic's hidden pre-activations z [2 n_rows, ld] (rows [0, n) = truncation slots, [n, 2n) = last-step
// observations) instead of by a separate value-head launch (K14 MODE 2) whose output the scan then loads.
// V = sum_j act(z_j) w_j + b with K14's arithmetic bit for bit: virtual lane j (of K14's 64) owns columns
// [4j, 4j + 4) and the sum runs K14's xor butterfly 32, 16, ..., 1 — lane sl of an L-lane row segment holds
// virtual lanes sl + k L (k < 64 / L), so steps o >= L are in-lane and o < L cross lanes (ds_swizzle).
template <int SEG_LOG2, int COMPACT, int VACT = -1>
__global__ __launch_bounds__(256) void gae_dpp_kernel(const float *__restrict__ rew, const float *__restrict__ val,
                                                      const float *__restrict__ term,
                                                      const uint8_t *__restrict__ closed,
                                                      const float *__restrict__ boot, int64_t n_rows, int T,
                                                      float gamma, float gl, int use_gae, float *__restrict__ adv,
                                                      float *__restrict__ ret, int *__restrict__ slot_t,
                                                      const float *__restrict__ vboot, float *__restrict__ boot_out,
                                                      const float *__restrict__ zc = nullptr, int64_t ldz = 0,
                                                      float slope = 0.f, const float *__restrict__ wc = nullptr,
                                                      const float *__restrict__ bc = nullptr) {
    constexpr bool VALUE = VACT >= 0;
    static_assert(!VALUE || COMPACT, "the value-fused scan is a compact-closure form");
    constexpr int L = 1 << SEG_LOG2;
    constexpr int C = 4 * L;
    const int lane = threadIdx.x & 63;
    const int sl = lane & (L - 1);
    const int seg_base = lane & ~(L - 1);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t row = wave * (64 / L) + (lane >> SEG_LOG2);
    const bool row_ok = row < n_rows;
    const int64_t base = row_ok ? row * (int64_t)T : 0;
    const int nchunks = (T + C - 1) / C;
    const uint64_t seg_mask = (L == 64) ? ~0ull : ((1ull << L) - 1ull);

    int st = -1;
    float vs = 0.f, vl = 0.f;
    constexpr int KV = VALUE ? 64 / L : 1;
    float4 zs[KV], zl[KV], wv[KV];
    float bias = 0.f;
    if constexpr (VALUE) {
        // every load unconditional from a clamped address (no branch whose join would wait for them all)
        const int64_t rs = row_ok ? row : 0;
        st = slot_t[rs];
        if (!row_ok) st = -1;
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int col = 4 * (sl + k * L);
            zs[k] = *reinterpret_cast<const float4 *>(zc + rs * ldz + col);
            zl[k] = *reinterpret_cast<const float4 *>(zc + (n_rows + rs) * ldz + col);
            wv[k] = *reinterpret_cast<const float4 *>(wc + col);
        }
        bias = bc[0];
    } else if (COMPACT && row_ok) {
        st = slot_t[row];
        vs = vboot[row];
        vl = vboot[n_rows + row];
    }
    float carry = 0.f, carry_v = 0.f;
    bool carry_any = false;
    bool has_last = false;   // this lane owns step T - 1 of its row (compact form)
    float last_boot = 0.f;
    for (int c = nchunks - 1; c >= 0; --c) {
        const int t0 = c * C + (L - 1 - sl) * 4;
        const bool in = row_ok && t0 < T;  // T % 4 == 0: a lane's 4 steps are all in or all out
        float r[4] = {0.f, 0.f, 0.f, 0.f}, v[4] = {0.f, 0.f, 0.f, 0.f}, d[4] = {0.f, 0.f, 0.f, 0.f};
        float bt[4] = {0.f, 0.f, 0.f, 0.f};
        bool cl[4] = {false, false, false, false};
        if constexpr (VALUE) {
            // unconditional loads (clamped step), validity by selects; then V(slot), V(last) from z
            const int64_t o = base + (in ? t0 : 0);
            const float4 r4 = ld4<1>(rew + o);
            const float4 v4 = ld4<1>(val + o);
            const float4 d4 = ld4<1>(term + o);
            if (c == nchunks - 1) {
                float ps[KV], pl[KV];
#pragma unroll
                for (int k = 0; k < KV; ++k) {
                    ps[k] = xpa_dot4(xpa_act4<VACT>(zs[k], slope), wv[k]);
                    pl[k] = xpa_dot4(xpa_act4<VACT>(zl[k], slope), wv[k]);
                }
#pragma unroll
                for (int m = KV / 2; m >= 1; m >>= 1)  // butterfly steps o = m L >= L: in-lane
#pragma unroll
                    for (int k = 0; k < KV; ++k)
                        if (k < (k ^ m)) {
                            const float a0 = ps[k] + ps[k ^ m], b0 = pl[k] + pl[k ^ m];
                            ps[k] = ps[k ^ m] = a0;
                            pl[k] = pl[k ^ m] = b0;
                        }
                float xs = ps[0], xl = pl[0];
                if constexpr (L == 64) {
                    xs += __shfl_xor(xs, 32, 64);
                    xl += __shfl_xor(xl, 32, 64);
                }
                if constexpr (L >= 32) { xs += swz_xor<16>(xs); xl += swz_xor<16>(xl); }
                xs += swz_xor<8>(xs); xl += swz_xor<8>(xl);
                xs += swz_xor<4>(xs); xl += swz_xor<4>(xl);
                xs += swz_xor<2>(xs); xl += swz_xor<2>(xl);
                xs += swz_xor<1>(xs); xl += swz_xor<1>(xl);
                vs = xs + bias;
                vl = xl + bias;
            }
            if (in) {
                r[0] = r4.x; r[1] = r4.y; r[2] = r4.z; r[3] = r4.w;
                v[0] = v4.x; v[1] = v4.y; v[2] = v4.z; v[3] = v4.w;
                d[0] = d4.x; d[1] = d4.y; d[2] = d4.z; d[3] = d4.w;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int t = t0 + e;
                    const bool lt = (t == T - 1);
                    cl[e] = lt || d[e] != 0.f || t == st;
                    bt[e] = lt ? (d[e] != 0.f ? 0.f : vl) : (t == st ? vs : 0.f);
                }
                if (t0 + 3 == T - 1) {
                    has_last = true;
                    last_boot = bt[3];
                }
            }
        } else if (in) {
            const float4 r4 = ld4<1>(rew + base + t0);
            const float4 v4 = ld4<1>(val + base + t0);
            const float4 d4 = ld4<1>(term + base + t0);
            r[0] = r4.x; r[1] = r4.y; r[2] = r4.z; r[3] = r4.w;
            v[0] = v4.x; v[1] = v4.y; v[2] = v4.z; v[3] = v4.w;
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z; d[3] = d4.w;
            if (COMPACT) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int t = t0 + e;
                    const bool lt = (t == T - 1);
                    cl[e] = lt || d[e] != 0.f || t == st;
                    bt[e] = lt ? (d[e] != 0.f ? 0.f : vl) : (t == st ? vs : 0.f);
                }
                if (t0 + 3 == T - 1) {
                    has_last = true;
                    last_boot = bt[3];
                }
            } else {
                const uint32_t c4 = *reinterpret_cast<const uint32_t *>(closed + base + t0);
                const float4 q4 = ld4<1>(boot + base + t0);
                bt[0] = q4.x; bt[1] = q4.y; bt[2] = q4.z; bt[3] = q4.w;
                cl[0] = (c4 & 0xff) != 0; cl[1] = ((c4 >> 8) & 0xff) != 0;
                cl[2] = ((c4 >> 16) & 0xff) != 0; cl[3] = (c4 >> 24) != 0;
            }
        }
        // v_{t+1} of this lane's last step = v[0] of the lane below it (it owns the following steps)
        float vn = dpp_mov<kDppWaveShr1>(0.f, v[0]);
        if (sl == 0) vn = carry_v;
        float a[4], b[4], adv_direct[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float vnext = (e < 3) ? v[e + 1] : vn;
            const float nv = cl[e] ? bt[e] : vnext;
            const float nd = 1.0f - d[e];
            if (use_gae) {
                b[e] = r[e] + gamma * nd * nv - v[e];
                a[e] = cl[e] ? 0.f : gl * nd;
            } else {
                b[e] = r[e] + (cl[e] ? gamma * bt[e] : 0.f);
                a[e] = cl[e] ? 0.f : gamma;
            }
            adv_direct[e] = r[e] + gamma * nv - v[e];
            if (!in) { a[e] = 1.f; b[e] = 0.f; }
        }
        float LA = 1.f, LB = 0.f;
        bool lany = false;
#pragma unroll
        for (int e = 3; e >= 0; --e) {
            LB = b[e] + a[e] * LB;
            LA = a[e] * LA;
            lany |= cl[e];
        }
        // inclusive scan in lane order inside the segment (lower lanes = later steps)
        dpp_combine<1, kDppRowShr + 1, 0xf>(LA, LB);
        dpp_combine<2, kDppRowShr + 2, 0xf>(LA, LB);
        dpp_combine<4, kDppRowShr + 4, 0xf>(LA, LB);
        dpp_combine<8, kDppRowShr + 8, 0xf>(LA, LB);
        if (L >= 32) dpp_combine<16, kDppRowBcast15, 0xa>(LA, LB);
        if (L == 64) dpp_combine<32, kDppRowBcast31, 0xc>(LA, LB);
        const float first = LB + LA * carry;  // A (or R) at this lane's first step
        const uint64_t segbits = (__ballot(lany) >> seg_base) & seg_mask;
        bool nany = carry_any || (segbits & ((1ull << sl) - 1ull)) != 0;
        float nxt = dpp_mov<kDppWaveShr1>(0.f, first);
        if (sl == 0) nxt = carry;
        float oa[4], orr[4];
        bool wr[4];
#pragma unroll
        for (int e = 3; e >= 0; --e) {
            const float x = b[e] + a[e] * nxt;
            const bool anyc = cl[e] || nany;
            oa[e] = use_gae ? x : adv_direct[e];
            orr[e] = use_gae ? x + v[e] : x;
            wr[e] = anyc && in;
            nxt = x;
            nany = anyc;
        }
        if (wr[0] && wr[1] && wr[2] && wr[3]) {
            st4<1>(adv + base + t0, make_float4(oa[0], oa[1], oa[2], oa[3]));
            st4<1>(ret + base + t0, make_float4(orr[0], orr[1], orr[2], orr[3]));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (wr[e]) {
                    adv[base + t0 + e] = oa[e];
                    ret[base + t0 + e] = orr[e];
                }
        }
        if (c > 0) {  // the earlier chunk continues from this chunk's first step (lane L-1)
            carry = __shfl(first, L - 1, L);
            carry_v = __shfl(v[0], L - 1, L);
            carry_any = carry_any || segbits != 0;
        } else if (COMPACT) {
            // xpa_rollout_bootstrap_fixup's writes (both bootstraps, slot reset), issued inside the loop where
            // st / vs / vl are known to have landed, the last step's bootstrap from the registers of the lane
            // that owns step T - 1.  (After the loop, re-reading term[T - 1] cost a dependent load whose
            // vmcnt(0) also waited for every adv/ret store of the wave, then one more HBM round trip.)
            if (has_last) boot_out[base + T - 1] = last_boot;
            if (row_ok && sl == 0) {
                int sw = st;
                asm volatile("" : "+v"(sw));  // keeps the slot address math here: hoisted out of the loop it
                                              // made every wave wait for slot_t before issuing r / v / d
                if (sw >= 0 && sw < T - 1) boot_out[base + sw] = vs;
                if (sw >= 0) slot_t[row] = -1;
            }
        }
    }
}

template <int COMPACT>
bool launch_gae_dpp(int seg_log2, dim3 grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, const float *rew,
                    const float *val, const float *term, const uint8_t *closed, const float *boot, int64_t n_envs,
                    int T, float gamma, float gl, int use_gae, float *adv, float *ret, int *slot_t,
                    const float *vboot, float *boot_out) {
#define XPA_GAE_DPP(S_)                                                                                              \
    do {                                                                                                             \
        if (e0 || e1)                                                                                                \
            hipExtLaunchKernelGGL((gae_dpp_kernel<S_, COMPACT>), grid, dim3(256), 0, s, e0, e1, 0, rew, val, term,    \
                                  closed, boot, n_envs, T, gamma, gl, use_gae, adv, ret, slot_t, vboot, boot_out,    \
                                  (const float *)nullptr, (int64_t)0, 0.f, (const float *)nullptr,                   \
                                  (const float *)nullptr);                                                           \
        else                                                                                                         \
            hipLaunchKernelGGL((gae_dpp_kernel<S_, COMPACT>), grid, dim3(256), 0, s, rew, val, term, closed, boot,    \
                               n_envs, T, gamma, gl, use_gae, adv, ret, slot_t, vboot, boot_out,                     \
                               (const float *)nullptr, (int64_t)0, 0.f, (const float *)nullptr,                      \
                               (const float *)nullptr);                                                              \
    } while (0)
    switch (seg_log2) {
        case 4: XPA_GAE_DPP(4); return true;
        case 5: XPA_GAE_DPP(5); return true;
        case 6: XPA_GAE_DPP(6); return true;
        default: return false;
    }
#undef XPA_GAE_DPP
}
}  // namespace

XPA_API int xpa_abi_version(void) { return XPA_ABI_VERSION; }

namespace {
__global__ __launch_bounds__(64) void dispatch_floor_kernel(float *p) {
    if (p) p[threadIdx.x] = 0.f;
}
}  // namespace

// An empty one-wave launch timed by the same dispatch-attached events as xpa_gae_scan_timed: the fixed
// cost (dispatch, cache fences, timestamps) that every launch carries on this clock, whatever its grid
// (flat 4.1-4.2 us for 1 x 64 up to 2048 x 1024 threads on MI355X, tools/gae_floor.hip, r01).
XPA_API int xpa_dispatch_floor_timed(void *ev_start, void *ev_stop, xpa_stream_t stream) {
    if (!ev_start != !ev_stop) return (int)hipErrorInvalidValue;
    if (!ev_start)  // no events: a plain empty launch (for other clocks)
        hipLaunchKernelGGL(dispatch_floor_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (float *)nullptr);
    else
        hipExtLaunchKernelGGL(dispatch_floor_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                              (hipEvent_t)ev_stop, 0, (float *)nullptr);
    return xpa_launch_status();
}

namespace {
__global__ __launch_bounds__(256) void stream_copy_kernel(const f4v *__restrict__ r, const f4v *__restrict__ v,
                                                          const f4v *__restrict__ d, f4v *__restrict__ a,
                                                          f4v *__restrict__ o, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4v x = __builtin_nontemporal_load(r + i);
    const f4v y = __builtin_nontemporal_load(v + i);
    const f4v z = __builtin_nontemporal_load(d + i);
    __builtin_nontemporal_store(x + y * z, a + i);
    __builtin_nontemporal_store(x * y + z, o + i);
}
}  // namespace

// Measurement aid: K1's algorithmic traffic with no scan — three 16-B streaming loads and two 16-B
// streaming stores per 4 elements (20 B per element) — timed by the same dispatch-attached events.
XPA_API int xpa_stream_copy_timed(const float *r, const float *v, const float *d, float *a, float *o, int64_t n,
                                  void *ev_start, void *ev_stop, xpa_stream_t stream) {
    if (n <= 0 || n % 4 || !r || !v || !d || !a || !o || !ev_start || !ev_stop) return (int)hipErrorInvalidValue;
    if (((uintptr_t)r | (uintptr_t)v | (uintptr_t)d | (uintptr_t)a | (uintptr_t)o) % 16) return (int)hipErrorInvalidValue;
    const int64_t n4 = n / 4;
    hipExtLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                          (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, (const f4v *)r, (const f4v *)v, (const f4v *)d,
                          (f4v *)a, (f4v *)o, n4);
    return xpa_launch_status();
}

namespace {
template <int VEC, int NT>
void launch_gae(dim3 grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, const float *rew, const float *val,
                const float *term, const uint8_t *closed, const float *boot, int64_t n_envs, int T, int seg_log2,
                float gamma, float gl, int use_gae, float *adv, float *ret) {
    if (e0 || e1)  // events recorded by the dispatch itself: the kernel's own start / end
        hipExtLaunchKernelGGL((gae_scan_kernel<VEC, NT>), grid, dim3(256), 0, s, e0, e1, 0, rew, val, term, closed,
                              boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret, (int *)nullptr,
                              (const float *)nullptr, (float *)nullptr);
    else
        hipLaunchKernelGGL((gae_scan_kernel<VEC, NT>), grid, dim3(256), 0, s, rew, val, term, closed, boot, n_envs, T,
                           seg_log2, gamma, gl, use_gae, adv, ret, (int *)nullptr, (const float *)nullptr,
                           (float *)nullptr);
}
}  // namespace

XPA_API int xpa_gae_scan(const float *rew, const float *val, const float *term, const uint8_t *closed,
                         const float *boot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                         int use_gae, float *adv, float *ret, xpa_stream_t stream) {
    return xpa_gae_scan_timed(rew, val, term, closed, boot, n_envs, horizon, gamma, gae_lambda, use_gae, adv, ret,
                              nullptr, nullptr, stream);
}

XPA_API int xpa_gae_scan_timed(const float *rew, const float *val, const float *term, const uint8_t *closed,
                               const float *boot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                               int use_gae, float *adv, float *ret, void *ev_start, void *ev_stop,
                               xpa_stream_t stream) {
    if (n_envs < 0 || horizon < 0 || horizon > (1 << 30)) return (int)hipErrorInvalidValue;
    if (n_envs == 0 || horizon == 0) return 0;
    if (!rew || !val || !term || !closed || !boot || !adv || !ret) return (int)hipErrorInvalidValue;
    const int T = (int)horizon;
    const bool vec4 = (T % 4 == 0) && ((uintptr_t)rew % 16 == 0) && ((uintptr_t)val % 16 == 0) &&
                      ((uintptr_t)term % 16 == 0) && ((uintptr_t)boot % 16 == 0) && ((uintptr_t)adv % 16 == 0) &&
                      ((uintptr_t)ret % 16 == 0) &&
                      ((uintptr_t)closed % 4 == 0);
    const int VEC = vec4 ? 4 : 1;
    int per_lane = (T + VEC - 1) / VEC;
    int seg_log2 = 0;
    while ((1 << seg_log2) < per_lane && seg_log2 < 6) ++seg_log2;
    const int64_t rows_per_wave = 64 >> seg_log2;
    const int64_t waves = (n_envs + rows_per_wave - 1) / rows_per_wave;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const float gl = gamma * gae_lambda;
    // Streaming (non-temporal) 16-B accesses: every byte is touched once.  Flushed sweep (r01, MI355X):
    // 65 536 x 128: 2.82 -> 4.26 TB/s, 262 144: 4.03 -> 5.02, 1 M: 4.97 -> 5.24 with nt.
    // XPA_GAE_NT=0 forces the plain form (A/B measurement).
    static const int nt_env = [] {
        const char *e = getenv("XPA_GAE_NT");
        return e ? atoi(e) : -1;
    }();
    const bool nt = nt_env != 0;
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    const dim3 grid((unsigned)blocks);
    static const int dpp_env = [] {
        const char *e = getenv("XPA_GAE_DPP");
        return e ? atoi(e) : -1;
    }();
    if (vec4 && nt && dpp_env != 0 &&
        launch_gae_dpp<0>(seg_log2, grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, gamma, gl, use_gae, adv,
                          ret, nullptr, nullptr, nullptr))
        return xpa_launch_status();
    if (vec4 && nt)
        launch_gae<4, 1>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    else if (vec4)
        launch_gae<4, 0>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    else
        launch_gae<1, 0>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    return xpa_launch_status();
}

XPA_API int xpa_gae_scan_compact(const float *rew, const float *val, const float *term, int32_t *slot_t,
                                 const float *vboot, int64_t n_envs, int64_t horizon, float gamma, float gae_lambda,
                                 int use_gae, float *adv, float *ret, float *boot, void *ev_start, void *ev_stop,
                                 xpa_stream_t stream) {
    if (n_envs < 0 || horizon < 0 || horizon > (1 << 30)) return (int)hipErrorInvalidValue;
    if (n_envs == 0 || horizon == 0) return 0;
    if (!rew || !val || !term || !slot_t || !vboot || !adv || !ret || !boot) return (int)hipErrorInvalidValue;
    const int T = (int)horizon;
    const bool vec4 = (T % 4 == 0) && ((uintptr_t)rew % 16 == 0) && ((uintptr_t)val % 16 == 0) &&
                      ((uintptr_t)term % 16 == 0) && ((uintptr_t)adv % 16 == 0) && ((uintptr_t)ret % 16 == 0);
    const int VEC = vec4 ? 4 : 1;
    const int per_lane = (T + VEC - 1) / VEC;
    int seg_log2 = 0;
    while ((1 << seg_log2) < per_lane && seg_log2 < 6) ++seg_log2;
    const int64_t rows_per_wave = 64 >> seg_log2;
    const int64_t blocks = ((n_envs + rows_per_wave - 1) / rows_per_wave + 3) / 4;
    if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const float gl = gamma * gae_lambda;
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    const dim3 grid((unsigned)blocks);
#define XPA_GAEC(V_, NT_)                                                                                            \
    do {                                                                                                             \
        if (e0 || e1)                                                                                                \
            hipExtLaunchKernelGGL((gae_scan_kernel<V_, NT_, 1>), grid, dim3(256), 0, s, e0, e1, 0, rew, val, term,     \
                                  (const uint8_t *)nullptr, (const float *)nullptr, n_envs, T, seg_log2, gamma, gl,  \
                                  use_gae, adv, ret, slot_t, vboot, boot);                                           \
        else                                                                                                         \
            hipLaunchKernelGGL((gae_scan_kernel<V_, NT_, 1>), grid, dim3(256), 0, s, rew, val, term,                   \
                               (const uint8_t *)nullptr, (const float *)nullptr, n_envs, T, seg_log2, gamma, gl,     \
                               use_gae, adv, ret, slot_t, vboot, boot);                                              \
    } while (0)
    static const int dpp_env = [] {
        const char *e = getenv("XPA_GAE_DPP");
        return e ? atoi(e) : -1;
    }();
    if (vec4 && dpp_env != 0 &&
        launch_gae_dpp<1>(seg_log2, grid, s, e0, e1, rew, val, term, nullptr, nullptr, n_envs, T, gamma, gl, use_gae,
                          adv, ret, slot_t, vboot, boot))
        return xpa_launch_status();
    if (vec4) XPA_GAEC(4, 1);
    else XPA_GAEC(1, 0);
#undef XPA_GAEC
    return xpa_launch_status();
}

namespace {
template <int S_, int A_>
void launch_gae_value(dim3 grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, const float *rew, const float *val,
                      const float *term, int64_t n_envs, int T, float gamma, float gl, int use_gae, float *adv,
                      float *ret, int *slot_t, float *boot, const float *z, int64_t ld, float slope, const float *w,
                      const float *b) {
    if (e0 || e1)
        hipExtLaunchKernelGGL((gae_dpp_kernel<S_, 1, A_>), grid, dim3(256), 0, s, e0, e1, 0, rew, val, term,
                              (const uint8_t *)nullptr, (const float *)nullptr, n_envs, T, gamma, gl, use_gae, adv, ret,
                              slot_t, (const float *)nullptr, boot, z, ld, slope, w, b);
    else
        hipLaunchKernelGGL((gae_dpp_kernel<S_, 1, A_>), grid, dim3(256), 0, s, rew, val, term, (const uint8_t *)nullptr,
                           (const float *)nullptr, n_envs, T, gamma, gl, use_gae, adv, ret, slot_t,
                           (const float *)nullptr, boot, z, ld, slope, w, b);
}
}  // namespace

XPA_API int xpa_gae_scan_value(const float *rew, const float *val, const float *term, int32_t *slot_t, int act,
                               const float *z_critic, int64_t ld, float slope, const float *w_critic,
                               const float *b_critic, int64_t n_envs, int64_t horizon, int64_t hidden, float gamma,
                               float gae_lambda, int use_gae, float *adv, float *ret, float *boot, void *ev_start,
                               void *ev_stop, xpa_stream_t stream) {
    if (n_envs <= 0 || horizon < 36 || horizon > (1 << 30) || horizon % 4 || hidden != 256 || ld < 256 || ld % 4 ||
        act < 0 || act > 2)
        return (int)hipErrorInvalidValue;
    if (!rew || !val || !term || !slot_t || !z_critic || !w_critic || !b_critic || !adv || !ret || !boot)
        return (int)hipErrorInvalidValue;
    if (((uintptr_t)rew | (uintptr_t)val | (uintptr_t)term | (uintptr_t)adv | (uintptr_t)ret | (uintptr_t)z_critic |
         (uintptr_t)w_critic) % 16)
        return (int)hipErrorInvalidValue;
    const int T = (int)horizon;
    int seg_log2 = 0;
    while ((1 << seg_log2) < T / 4 && seg_log2 < 6) ++seg_log2;  // T >= 36: seg_log2 in [4, 6]
    const int64_t rows_per_wave = 64 >> seg_log2;
    const int64_t blocks = ((n_envs + rows_per_wave - 1) / rows_per_wave + 3) / 4;
    if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)blocks);
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    const float gl = gamma * gae_lambda;
#define XPA_GAEV(S_, A_)                                                                                        \
    launch_gae_value<S_, A_>(grid, s, e0, e1, rew, val, term, n_envs, T, gamma, gl, use_gae, adv, ret, slot_t, boot, \
                             z_critic, ld, slope, w_critic, b_critic)
#define XPA_GAEV_ACT(S_)             \
    do {                             \
        if (act == 0) XPA_GAEV(S_, 0); \
        else if (act == 1) XPA_GAEV(S_, 1); \
        else XPA_GAEV(S_, 2);        \
    } while (0)
    switch (seg_log2) {
        case 4: XPA_GAEV_ACT(4); break;
        case 5: XPA_GAEV_ACT(5); break;
        default: XPA_GAEV_ACT(6); break;
    }
#undef XPA_GAEV_ACT
#undef XPA_GAEV
    return xpa_launch_status();
}
