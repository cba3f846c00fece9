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

template <int VEC, int NT>
__global__ __launch_bounds__(256) void gae_scan_kernel(const float *__restrict__ rew, const float *__restrict__ val,
                                                       const float *__restrict__ term,
                                                       const uint8_t *__restrict__ closed,
                                                       const float *__restrict__ boot, int64_t n_rows, int T,
                                                       int seg_log2, float gamma, float gl, int use_gae,
                                                       float *__restrict__ adv, float *__restrict__ ret) {
    const int L = 1 << seg_log2;
    const int lane = threadIdx.x & 63;
    const int sl = lane & (L - 1);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t row = wave * (64 >> seg_log2) + (lane >> seg_log2);
    const bool row_ok = row < n_rows;
    const int64_t base = row_ok ? row * (int64_t)T : 0;
    const int C = L * VEC;
    const int nchunks = (T + C - 1) / C;

    float carry = 0.f;   // A (or R) at the first element of the later chunk
    float carry_v = 0.f; // v at that element
    int carry_any = 0;   // a closure exists at or after the later chunk's first element

    for (int c = nchunks - 1; c >= 0; --c) {
        const int t0 = c * C + sl * VEC;
        float r[VEC], v[VEC], d[VEC], bt[VEC];
        int cl[VEC];
        const bool full = row_ok && (t0 + VEC <= T);
        if (VEC == 4 && full) {
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
    if (!ev_start || !ev_stop) return (int)hipErrorInvalidValue;
    hipExtLaunchKernelGGL(dispatch_floor_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                          (hipEvent_t)ev_stop, 0, (float *)nullptr);
    return xpa_launch_status();
}

namespace {
template <int VEC, int NT>
void launch_gae(dim3 grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, const float *rew, const float *val,
                const float *term, const uint8_t *closed, const float *boot, int64_t n_envs, int T, int seg_log2,
                float gamma, float gl, int use_gae, float *adv, float *ret) {
    if (e0 || e1)  // events recorded by the dispatch itself: the kernel's own start / end
        hipExtLaunchKernelGGL((gae_scan_kernel<VEC, NT>), grid, dim3(256), 0, s, e0, e1, 0, rew, val, term, closed,
                              boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    else
        hipLaunchKernelGGL((gae_scan_kernel<VEC, NT>), grid, dim3(256), 0, s, rew, val, term, closed, boot, n_envs, T,
                           seg_log2, gamma, gl, use_gae, adv, ret);
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
    if (vec4 && nt)
        launch_gae<4, 1>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    else if (vec4)
        launch_gae<4, 0>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    else
        launch_gae<1, 0>(grid, s, e0, e1, rew, val, term, closed, boot, n_envs, T, seg_log2, gamma, gl, use_gae, adv, ret);
    return xpa_launch_status();
}
