// K15 — SynthAtari env step on device (the Atari-shaped synthetic env of SURVEY.md §8(d), C3 / C5).
//
// Replaces, for the benchmark, DummyVecEnv_Atari stepping Atari_Env (xuance/environment/gym/
// gym_vec_env.py:201-212, 234-238; gym_env.py:186-241): uint8 [84, 84, 4] HWC frame stacks, reward
// sign, life-loss / game-over flags, auto-reset with reset_obs.  Spec and CPU checker:
// oracle/synth_env.py (SynthAtariEnv) — bit-identical frames, rewards and flags.
//
// Layout: the stack of env n is [84*84] uint32 (4 channels of a pixel = one dword, channel 3 = newest),
// so pushing a frame is `stack = (stack >> 8) | (pixel << 24)` per pixel: 28 KiB read + 2 x 28 KiB
// written per env step (the stepped stack as final_obs, the next observation).
// One block per env: thread 0 advances the scalar state, the block renders the frame.
#include "xpa_common.h"

namespace {

constexpr int kHW = 84;
constexpr int kPix = kHW * kHW;
constexpr int kLives = 5;
constexpr int kPx0 = 38;
constexpr uint32_t kSaltPix = 0xA7A21000u;
constexpr uint32_t kSaltBall = 0xBA11B000u;

__device__ __forceinline__ uint32_t ball_x(uint32_t seed, uint32_t env, uint32_t ep, uint32_t t) {
    return xpa_hash4(seed ^ kSaltBall, env, ep, t >> 4) % 77u;
}

// pixel p of frame(ep, t, px); pre = mix32(mix32(mix32(seed ^ kSaltPix) ^ env) ^ ep) (the per-episode
// prefix of the background hash)
__device__ __forceinline__ uint32_t frame_pixel(uint32_t pre, int p, int bx, int by, int px) {
    const int y = p / kHW, x = p - y * kHW;
    uint32_t v = xpa_mix32(pre ^ (uint32_t)p) >> 27;
    if (y >= by && y < by + 8 && x >= bx && x < bx + 8) v = 255u;
    if (y >= 78 && y < 82 && x >= px && x < px + 8) v = 200u;
    return v;
}

__device__ __forceinline__ uint32_t ep_prefix(uint32_t seed, uint32_t env, uint32_t ep) {
    return xpa_mix32(xpa_mix32(xpa_mix32(seed ^ kSaltPix) ^ env) ^ ep);
}

__global__ __launch_bounds__(256) void synthatari_step_kernel(
    int K, const float *__restrict__ act_in, int64_t ld_act, uint32_t seed, int max_steps,
    uint32_t *__restrict__ stack, uint32_t *__restrict__ final_obs, float *__restrict__ rew,
    uint8_t *__restrict__ term, uint8_t *__restrict__ trunc, int *__restrict__ ep_step, int *__restrict__ ep_index,
    int *__restrict__ lives, int *__restrict__ pxs, float *__restrict__ ep_score, float *__restrict__ ep_last_score,
    int *__restrict__ ep_last_len, int *__restrict__ err) {
    __shared__ int s_px, s_t, s_over, s_bx, s_by, s_bx0, s_by0;
    __shared__ uint32_t s_pre, s_pre0;
    const int64_t n = blockIdx.x;
    const uint32_t env = (uint32_t)n;
    if (threadIdx.x == 0) {
        int a = -1;  // the env input is the one-hot written by the sampler
        for (int k = 0; k < K; ++k)
            if (act_in[n * ld_act + k] > 0.5f) {
                a = k;
                break;
            }
        if (a < 0) {  // no action set: NOOP, counted
            if (err) atomicAdd(err, 1);
            a = 0;
        }
        const uint32_t ep = (uint32_t)ep_index[n];
        const int t = ep_step[n];
        int px = pxs[n] + ((a + 1) % 3 - 1) * 3;
        px = px < 0 ? 0 : (px > 76 ? 76 : px);
        float r = 0.f;
        if ((t & 15) == 15) r = (abs(px - (int)ball_x(seed, env, ep, (uint32_t)t)) <= 8) ? 1.f : -1.f;
        const int t1 = t + 1;
        const float score = ep_score[n] + r;
        int lv = lives[n] - (r < 0.f ? 1 : 0);
        const bool over = lv == 0 || t1 >= max_steps;
        rew[n] = r;
        term[n] = (over || r < 0.f) ? 1 : 0;
        trunc[n] = over ? 1 : 0;
        s_px = px;
        s_t = t1;
        s_over = over ? 1 : 0;
        s_pre = ep_prefix(seed, env, ep);
        s_bx = (int)ball_x(seed, env, ep, (uint32_t)t1);
        s_by = (t1 & 15) * 5;
        if (over) {
            ep_last_score[n] = score;
            ep_last_len[n] = t1;
            ep_index[n] = (int)(ep + 1u);
            ep_step[n] = 0;
            ep_score[n] = 0.f;
            lives[n] = kLives;
            pxs[n] = kPx0;
            s_pre0 = ep_prefix(seed, env, ep + 1u);
            s_bx0 = (int)ball_x(seed, env, ep + 1u, 0u);
            s_by0 = 0;
        } else {
            ep_step[n] = t1;
            ep_score[n] = score;
            lives[n] = lv;
            pxs[n] = px;
        }
    }
    __syncthreads();
    const int px = s_px, bx = s_bx, by = s_by, over = s_over;
    const uint32_t pre = s_pre;
    uint32_t *st = stack + n * kPix;
    uint32_t *fo = final_obs + n * kPix;
    for (int p = threadIdx.x; p < kPix; p += 256) {
        const uint32_t v = (st[p] >> 8) | (frame_pixel(pre, p, bx, by, px) << 24);
        fo[p] = v;
        st[p] = over ? frame_pixel(s_pre0, p, s_bx0, s_by0, kPx0) * 0x01010101u : v;
    }
}

__global__ __launch_bounds__(256) void synthatari_reset_kernel(uint32_t seed, uint32_t *__restrict__ stack,
                                                               const int *__restrict__ ep_index) {
    const int64_t n = blockIdx.x;
    const uint32_t ep = (uint32_t)ep_index[n];
    const uint32_t pre = ep_prefix(seed, (uint32_t)n, ep);
    const int bx = (int)ball_x(seed, (uint32_t)n, ep, 0u);
    for (int p = threadIdx.x; p < kPix; p += 256) stack[n * kPix + p] = frame_pixel(pre, p, bx, 0, kPx0) * 0x01010101u;
}

}  // namespace

XPA_API int xpa_synthatari_step(int64_t n_envs, int64_t n_actions, const float *act_in, int64_t ld_act, uint32_t seed,
                                int32_t max_episode_steps, uint8_t *stack, uint8_t *final_obs, float *rew,
                                uint8_t *term, uint8_t *trunc, int32_t *ep_step, int32_t *ep_index, int32_t *lives,
                                int32_t *paddle, float *ep_score, float *ep_last_score, int32_t *ep_last_len,
                                int32_t *err, xpa_stream_t stream) {
    if (n_envs <= 0 || n_envs > 0x7fffffff || n_actions < 1 || ld_act < n_actions || max_episode_steps <= 0 ||
        !act_in || !stack || !final_obs || !rew || !term || !trunc || !ep_step || !ep_index || !lives || !paddle ||
        !ep_score || !ep_last_score || !ep_last_len || ((uintptr_t)stack | (uintptr_t)final_obs) % 4)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(synthatari_step_kernel, dim3((unsigned)n_envs), dim3(256), 0, (hipStream_t)stream,
                       (int)n_actions, act_in, ld_act, seed, (int)max_episode_steps, (uint32_t *)stack,
                       (uint32_t *)final_obs, rew, term, trunc, ep_step, ep_index, lives, paddle, ep_score,
                       ep_last_score, ep_last_len, err);
    return xpa_launch_status();
}

XPA_API int xpa_synthatari_reset(int64_t n_envs, uint32_t seed, uint8_t *stack, const int32_t *ep_index,
                                 xpa_stream_t stream) {
    if (n_envs <= 0 || n_envs > 0x7fffffff || !stack || !ep_index || (uintptr_t)stack % 4)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(synthatari_reset_kernel, dim3((unsigned)n_envs), dim3(256), 0, (hipStream_t)stream, seed,
                       (uint32_t *)stack, ep_index);
    return xpa_launch_status();
}
