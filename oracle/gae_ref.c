/* ORACLE / TEST INFRASTRUCTURE — plain-C restatement of the reference's GAE/returns.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library
 * (oracle/_build/liboracle_gae.so).  It is the checker for the HIP kernel xpa_gae_scan, never
 * the product path.
 *
 * Follows /root/reference/xuance/common/memory_tools.py:206-229 (DummyOnPolicyBuffer.finish_path):
 *   vs = values[path] ++ [val]
 *   use_gae:  delta_t = r_t + (1-d_t) g vs[t+1] - vs[t];  A_t = delta_t + (1-d_t) g l A_{t+1};  R = A + v
 *   else:     R = discount_cumsum(r ++ [val], g)[:-1]  (no done mask, common_tools.py:199-200)
 *             A_t = r_t + g vs[t+1] - vs[t]
 * and the agent-side path closing of ppoclip_agent.py:69-101 / a2c_agent.py:66-98, expressed as
 * per-(env, step) closure flags: closed[n,t] = 1 when finish_path(boot[n,t], n) ended a path whose
 * last stored step is t.  Arithmetic in double (the reference mixes f32/f64 through NumPy
 * promotion); the GPU kernel computes in f32 and is compared within 1e-5.
 */
#include <stddef.h>
#include <stdint.h>

/* One call of finish_path over path [start, end) of one env row (memory_tools.py:206-229). */
void oracle_finish_path(const float *rew, const float *val, const float *term, int start, int end,
                        double bootstrap, double gamma, double lam, int use_gae, float *adv,
                        float *ret) {
    int n = end - start;
    if (n <= 0) return;
    if (use_gae) {
        double last = 0.0;
        for (int k = n - 1; k >= 0; --k) {
            int t = start + k;
            double vnext = (k == n - 1) ? bootstrap : (double)val[t + 1];
            double nd = 1.0 - (double)term[t];
            double delta = (double)rew[t] + nd * gamma * vnext - (double)val[t];
            last = delta + nd * gamma * lam * last;
            adv[t] = (float)last;
            ret[t] = (float)(last + (double)val[t]);
        }
    } else {
        double run = bootstrap; /* lfilter over reversed (r ++ [val]) */
        for (int k = n - 1; k >= 0; --k) {
            int t = start + k;
            double vnext = (k == n - 1) ? bootstrap : (double)val[t + 1];
            run = (double)rew[t] + gamma * run;
            ret[t] = (float)run;
            adv[t] = (float)((double)rew[t] + gamma * vnext - (double)val[t]);
        }
    }
}

/* Whole [n_envs, horizon] buffer: every row is cut into paths at its closure flags; a path ends at
 * step t when closed[n*T+t] != 0, with bootstrap boot[n*T+t].  Positions after the last closure of
 * a row (an open path) are left untouched, as in the reference. */
void oracle_gae_rows(const float *rew, const float *val, const float *term, const uint8_t *closed,
                     const float *boot, int n_envs, int horizon, double gamma, double lam,
                     int use_gae, float *adv, float *ret) {
    for (int n = 0; n < n_envs; ++n) {
        size_t o = (size_t)n * (size_t)horizon;
        int start = 0;
        for (int t = 0; t < horizon; ++t) {
            if (closed[o + t]) {
                oracle_finish_path(rew + o, val + o, term + o, start, t + 1, (double)boot[o + t],
                                   gamma, lam, use_gae, adv + o, ret + o);
                start = t + 1;
            }
        }
    }
}
