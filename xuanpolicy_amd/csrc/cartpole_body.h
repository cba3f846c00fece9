// CartPole-v1 per-env step (gym 0.26.2 classic_control/cartpole.py + TimeLimit), shared by K18
// (xpa_cartpole_step, classic.hip) and K32's fused rollout step (rollout.hip) so both run the same arithmetic.
#pragma once
#include "xpa_common.h"

struct XpaCartPoleEnv {
    double *state;  // [N, 4] f64 (x, x_dot, theta, theta_dot)
    float *obs;     // [N, ld_obs]: the next observation (the reset state after a done)
    int64_t ld_obs;
    float *final_obs;  // [N, 4]: the step's own observation (before any reset)
    float *rew;
    uint8_t *term, *trunc;
    int *ep_step;
    uint32_t *ep_index;
    float *ep_score, *ep_last_score;
    int *ep_last_len;
    uint32_t seed;
    int max_episode_steps;
    double theta_threshold;
};

namespace cartpole {
constexpr double kGravity = 9.8, kMassPole = 0.1, kTotalMass = 1.1, kLength = 0.5, kPoleMassLength = 0.05;
constexpr double kForce = 10.0, kTau = 0.02, kXThreshold = 2.4;
constexpr uint32_t kSaltCartPole = 0xCA27B01Eu;
constexpr double kThetaThreshold = 12.0 * 2.0 * 3.141592653589793 / 360.0;  // gym: 12 * 2 * math.pi / 360

__device__ __forceinline__ double reset_dim(uint32_t seed, uint32_t env, uint32_t ep, uint32_t d) {
    return (double)xpa_u01(xpa_hash4(seed ^ kSaltCartPole, env, ep, d)) * 0.1 - 0.05;
}

// One env's mutable state, held in registers by the caller (K18 loads and stores it around one step; K32 keeps it
// for a whole launch of steps).
struct Local {
    double x, x_dot, theta, theta_dot;
    int ep_step;
    uint32_t ep_index;
    float ep_score;
};

__device__ __forceinline__ Local load(const XpaCartPoleEnv &e, int64_t n) {
    const double *st = e.state + 4 * n;
    return Local{st[0], st[1], st[2], st[3], e.ep_step[n], e.ep_index[n], e.ep_score[n]};
}

__device__ __forceinline__ void store(const XpaCartPoleEnv &e, int64_t n, const Local &s) {
    double *st = e.state + 4 * n;
    st[0] = s.x;
    st[1] = s.x_dot;
    st[2] = s.theta;
    st[3] = s.theta_dot;
    e.ep_step[n] = s.ep_step;
    e.ep_index[n] = s.ep_index;
    e.ep_score[n] = s.ep_score;
}

// One env's step with action a (0 / 1) on the register state s: writes final_obs / obs / rew / term / trunc (and
// the finished episode's score / length); returns the reward, *te / *tr the flags, obs_out[0..3] the next
// observation (the reset state after a done).
__device__ __forceinline__ float step(const XpaCartPoleEnv &e, int64_t n, int a, Local &s, bool *te_out,
                                      bool *tr_out, float *obs_out) {
#pragma clang fp contract(off)  // gym's Python arithmetic: every product and sum rounded on its own (no fma)
    double x = s.x, x_dot = s.x_dot, theta = s.theta, theta_dot = s.theta_dot;
    const double force = a == 1 ? kForce : -kForce;
    const double costheta = cos(theta), sintheta = sin(theta);
    const double temp = (force + kPoleMassLength * (theta_dot * theta_dot) * sintheta) / kTotalMass;
    const double thetaacc = (kGravity * sintheta - costheta * temp) /
                            (kLength * (4.0 / 3.0 - kMassPole * (costheta * costheta) / kTotalMass));
    const double xacc = temp - kPoleMassLength * thetaacc * costheta / kTotalMass;
    x = x + kTau * x_dot;
    x_dot = x_dot + kTau * xacc;
    theta = theta + kTau * theta_dot;
    theta_dot = theta_dot + kTau * thetaacc;
    const double th = e.theta_threshold;
    const bool te = x < -kXThreshold || x > kXThreshold || theta < -th || theta > th;
    const int steps = s.ep_step + 1;
    const bool tr = steps >= e.max_episode_steps;  // gym TimeLimit: independent of terminated
    const float score = s.ep_score + 1.0f;
    float *fo = e.final_obs + 4 * n;
    fo[0] = (float)x;
    fo[1] = (float)x_dot;
    fo[2] = (float)theta;
    fo[3] = (float)theta_dot;
    e.rew[n] = 1.0f;
    e.term[n] = te ? 1 : 0;
    e.trunc[n] = tr ? 1 : 0;
    if (te || tr) {
        const uint32_t ep = s.ep_index + 1u;
        s.ep_index = ep;
        e.ep_last_score[n] = score;
        e.ep_last_len[n] = steps;
        s.ep_step = 0;
        s.ep_score = 0.f;
        x = reset_dim(e.seed, (uint32_t)n, ep, 0);
        x_dot = reset_dim(e.seed, (uint32_t)n, ep, 1);
        theta = reset_dim(e.seed, (uint32_t)n, ep, 2);
        theta_dot = reset_dim(e.seed, (uint32_t)n, ep, 3);
    } else {
        s.ep_step = steps;
        s.ep_score = score;
    }
    s.x = x;
    s.x_dot = x_dot;
    s.theta = theta;
    s.theta_dot = theta_dot;
    obs_out[0] = (float)x;
    obs_out[1] = (float)x_dot;
    obs_out[2] = (float)theta;
    obs_out[3] = (float)theta_dot;
    float *o = e.obs + n * e.ld_obs;
    o[0] = obs_out[0];
    o[1] = obs_out[1];
    o[2] = obs_out[2];
    o[3] = obs_out[3];
    *te_out = te;
    *tr_out = tr;
    return 1.0f;
}
}  // namespace cartpole
