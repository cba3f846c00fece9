"""ctypes binding of the C ABI in include/xuanpolicy_amd.h (libxuanpolicy_amd.so, gfx950).

The library is built in-tree by `build_library()` (hipcc, --offload-arch=gfx950) and loaded after
`import torch`, so its NEEDED libamdhip64.so.7 resolves to the HIP runtime torch already mapped
(same SONAME) and torch's device pointers and hipStream_t handles are valid in it.

There is no CPU fallback: every entry point raises if the library is missing or a call fails.
"""
import ctypes
import os
import subprocess

import torch  # noqa: F401  (must be loaded first: see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libxuanpolicy_amd.so")
CSRC = os.path.join(PKG_DIR, "csrc")
SOURCES = ["gae.hip", "loss.hip", "rollout.hip", "optim.hip", "mlp.hip", "head.hip", "thin.hip", "per.hip", "atari.hip",
           "classic.hip", "dqn.hip", "conv.hip", "igemm.hip", "smallmlp.hip", "sgemm3.hip"]
HEADER = os.path.join(REPO_DIR, "include", "xuanpolicy_amd.h")

ABI_VERSION = 4
COLSUM_TICKET_INTS = 4096   # include/xuanpolicy_amd.h XPA_COLSUM_TICKET_INTS (ABI 4)

c_i32, c_i64, c_u32, c_f32, c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float, ctypes.c_void_p

class XpaSmallMlpArgs(ctypes.Structure):
    """include/xuanpolicy_amd.h XpaSmallMlpArgs (K30), field for field."""
    _fields_ = ([(n, ctypes.c_int) for n in ("batch", "d_in", "h0", "h1", "h2", "k", "act_code", "algo", "use_advnorm",
                                             "n_sched")]
                + [(n, ctypes.c_float) for n in ("slope", "clip_range", "vf_coef", "ent_coef", "max_norm", "beta1",
                                                 "beta2", "eps")]
                + [("obs", ctypes.c_void_p), ("obs_ld", ctypes.c_int64), ("idx", ctypes.c_void_p),
                   ("n_rows", ctypes.c_int64)]
                + [(n, ctypes.c_void_p) for n in ("actions", "old_logp", "adv", "ret", "W0", "b0", "W1", "b1", "W2",
                                                  "b2", "Wa", "ba", "Wc", "bc", "gW0", "gb0", "gW1", "gb1", "gW2",
                                                  "gb2", "gWa", "gba", "gWc", "gbc", "param", "grad", "exp_avg",
                                                  "exp_avg_sq")]
                + [("n", ctypes.c_int64), ("sched", ctypes.c_void_p), ("cursor", ctypes.c_void_p),
                   ("scalars", ctypes.c_void_p), ("total_norm_out", ctypes.c_void_p), ("stamps", ctypes.c_void_p),
                   ("n_groups", ctypes.c_int), ("grad_part", ctypes.c_void_p), ("loss_part", ctypes.c_void_p)])


class XpaSmallRolloutArgs(ctypes.Structure):
    """include/xuanpolicy_amd.h XpaSmallRolloutArgs (K32), field for field."""
    _fields_ = ([(n, ctypes.c_int) for n in ("n_envs", "horizon", "steps", "d_in", "h0", "h1", "h2", "k", "act_code",
                                             "use_obsnorm", "n_slots", "mask_returns", "use_rewnorm",
                                             "max_episode_steps", "slot_reset_obs")]
                + [(n, ctypes.c_float) for n in ("slope", "obs_clip", "gamma", "rew_range")]
                + [("seed", ctypes.c_uint32), ("env_seed", ctypes.c_uint32)]
                + [(n, ctypes.c_void_p) for n in ("W0", "b0", "W1", "b1", "W2", "b2", "Wa", "ba", "Wc", "bc",
                                                  "obs_mean", "obs_var", "obs_count", "obs_norm")]
                + [("ld_norm", ctypes.c_int64)]
                + [(n, ctypes.c_void_p) for n in ("buf_obs", "buf_act", "buf_logp", "buf_val", "buf_rew", "buf_term",
                                                  "buf_closed", "buf_boot", "act_in")]
                + [("ld_act", ctypes.c_int64), ("env_state", ctypes.c_void_p), ("env_obs", ctypes.c_void_p),
                   ("ld_obs", ctypes.c_int64)]
                + [(n, ctypes.c_void_p) for n in ("final_obs", "env_rew", "env_term", "env_trunc", "ep_step",
                                                  "ep_index", "ep_score", "ep_last_score", "ep_last_len", "returns",
                                                  "ret_mean", "ret_var", "ret_count", "slot_obs", "slot_t", "overflow",
                                                  "boot_norm")]
                + [("ld_boot", ctypes.c_int64), ("cursor", ctypes.c_void_p), ("stamps", ctypes.c_void_p)])


# name -> (restype, argtypes); mirrors include/xuanpolicy_amd.h one-for-one.
SIGNATURES = {
    "xpa_abi_version": (ctypes.c_int, []),
    "xpa_gae_scan": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, ctypes.c_int, c_p, c_p, c_p]),
    "xpa_gae_scan_compact": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, ctypes.c_int, c_p, c_p,
                                            c_p, c_p, c_p, c_p]),
    "xpa_gae_scan_value": (ctypes.c_int, [c_p, c_p, c_p, c_p, ctypes.c_int, c_p, c_i64, c_f32, c_p, c_p, c_i64, c_i64,
                                          c_i64, c_f32, c_f32, ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_stream_copy_timed": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p]),
    "xpa_gae_scan_timed": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, ctypes.c_int, c_p, c_p,
                                          c_p, c_p, c_p]),
    "xpa_dispatch_floor_timed": (ctypes.c_int, [c_p, c_p, c_p]),
    "xpa_random_permutation": (ctypes.c_int, [c_i64, c_u32, c_u32, c_p, c_p]),
    "xpa_gather_num_partials": (c_i64, [c_i64]),
    "xpa_gather_minibatch": (ctypes.c_int, [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p]),
    "xpa_loss_num_partials": (c_i64, [c_i64]),
    "xpa_loss_partial_width": (c_i64, [c_i64]),
    "xpa_policy_loss_fwd_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p,
                                               c_p, c_p, c_p, c_p, c_i64, c_f32, c_f32, c_f32, c_p, c_p, c_p, c_p]),
    "xpa_policy_loss_finalize": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_f32, c_f32,
                                                c_p, c_p, c_p]),
    "xpa_rms_num_partials": (c_i64, [c_i64]),
    "xpa_rms_partials": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "xpa_rms_update": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_rms_merge": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p]),
    "xpa_obs_normalize": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_i64, c_p, c_p]),
    "xpa_rollout_sample": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_u32, c_f32, c_p, c_p,
                                          c_p, c_p, c_i64, c_p]),
    "xpa_synthbox_step": (ctypes.c_int, [c_i64, c_i64, c_p, c_u32, c_i32, c_f32, c_f32, c_f32, c_p, c_i64, c_p, c_p,
                                         c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_cartpole_step": (ctypes.c_int, [c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                         c_p, c_u32, c_i32, c_p]),
    "xpa_dqn_td_loss": (ctypes.c_int, [c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p,
                                       c_p, c_p]),
    "xpa_rollout_post_num_blocks": (c_i64, [c_i64]),
    "xpa_rollout_post": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                        c_f32, ctypes.c_int, ctypes.c_int, c_f32, ctypes.c_int, c_p, c_p, c_p]),
    "xpa_act_bwd_num_partials": (c_i64, [c_i64]),
    "xpa_act_bwd_colsum": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_i64, c_i64, c_f32, c_p, c_p, c_p]),
    "xpa_colsum_finalize": (ctypes.c_int, [c_p, c_i64, c_i64, c_p, c_p]),
    "xpa_frames_to_f32": (ctypes.c_int, [c_p, c_i64, c_p, c_p]),
    "xpa_conv_dgrad_s2k": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64,
                                           c_i64, c_p, c_p]),
    "xpa_conv1_u8_wgrad_num_partials": (c_i64, []),
    "xpa_conv1_u8_wgrad_act": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_f32, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                               c_i64, c_i64, c_p, c_p, c_p]),
    "xpa_conv1_u8_wgrad": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "xpa_conv1_form": (ctypes.c_int, [ctypes.c_int]),
    "xpa_conv_igemm_form": (ctypes.c_int, [ctypes.c_int]),
    "xpa_conv1_u8_fwd": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p,
                                         c_i64, c_f32, c_p, c_p]),
    "xpa_bias_act": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_p, c_f32, c_p]),
    "xpa_act_bwd_bias_num_partials": (c_i64, [c_i64, c_i64]),
    "xpa_act_bwd_bias": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_i64, c_i64, c_f32, c_p, c_p, c_p]),
    "xpa_global_maxpool": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "xpa_maxpool_act_bwd_bias": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f32, c_p, c_p,
                                                c_p, c_p]),
    "xpa_head_bwd_num_partials": (c_i64, [c_i64]),
    "xpa_head_backward": (ctypes.c_int, [ctypes.c_int, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_f32, c_p, c_p, c_p,
                                         c_p, c_p]),
    "xpa_head_fused_num_partials": (c_i64, [c_i64]),
    "xpa_head_fused_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_i64, c_p, c_p,
                                            c_p,
                                            c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_f32, c_f32, c_p, c_p,
                                            c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_fused_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_f32, c_p, c_i64, c_p, c_f32,
                                             c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_rollout_policy_head": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p,
                                               c_f32, c_p, c_p, c_p, c_p, c_p, c_p, c_u32, c_f32, c_p, c_p, c_p, c_p,
                                               c_i64, c_p]),
    "xpa_rollout_policy_head_synthbox": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f32,
                                                        c_p, c_p, c_p, c_p, c_p, c_p, c_u32, c_f32, c_p, c_p, c_p,
                                                        c_i64, c_p, c_u32, ctypes.c_int32, c_f32, c_f32, c_f32, c_p,
                                                        c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_value_head": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p]),
    "xpa_colsum_batch_tiles": (c_i64, [ctypes.c_int, c_p, c_p]),
    "xpa_colsum_finalize_batch_sq": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_colsum_finalize_batch_sq_loss": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p, ctypes.c_int,
                                                         ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_f32, c_f32, c_p,
                                                         c_p, c_p]),
    "xpa_policy_loss_finalize_sq": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_f32, c_f32,
                                                   c_p, c_p, c_p, c_p]),
    "xpa_clip_adam_step_partials": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_f32, c_f32, c_f32, c_f32,
                                                   c_f32, c_i64, c_p, c_p]),
    "xpa_clip_adam_step_sched": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_p, c_f32, c_f32, c_f32, c_f32, c_p, c_i64,
                                                c_p, c_p, c_p]),
    "xpa_adam_sched_entry": (None, [c_f32, c_f32, c_f32, c_i64, c_p]),
    "xpa_small_mlp_lds_floats": (c_i64, [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "xpa_small_mlp_update": (ctypes.c_int, [c_p, c_p]),
    "xpa_small_rollout_lds_floats": (c_i64, [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "xpa_small_rollout_cartpole": (ctypes.c_int, [c_p, c_p]),
    "xpa_colsum_finalize_batch": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p]),
    "xpa_per_store": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i64, c_i64, ctypes.c_double, c_p]),
    "xpa_per_update_priorities": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_i64, ctypes.c_double,
                                                 c_p, c_p]),
    "xpa_per_sample": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_u32, c_u32, ctypes.c_double,
                                      ctypes.c_int, c_p, c_p, c_p, c_p, c_p]),
    "xpa_store_column": (ctypes.c_int, [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p]),
    "xpa_synthatari_step": (ctypes.c_int, [c_i64, c_i64, c_p, c_i64, c_u32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                           c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_synthatari_reset": (ctypes.c_int, [c_i64, c_u32, c_p, c_p, c_p]),
    "xpa_rollout_post_deferred_norm": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_i64, c_p,
                                                      c_p, c_f32,
                                                      c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                                      c_p, c_p, c_p, c_f32, ctypes.c_int, ctypes.c_int, c_f32,
                                                      ctypes.c_int, c_p, c_p, c_p]),
    "xpa_rollout_post_deferred": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_i64, c_p,
                                                 c_p, c_p,
                                                 c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32, ctypes.c_int, ctypes.c_int,
                                                 c_f32, ctypes.c_int, c_p, c_p, c_p]),
    "xpa_conv_igemm_ok": (ctypes.c_int, [c_i64, c_i64, c_i64]),
    "xpa_conv_fwd": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i64,
                                    c_f32, c_p, c_p]),
    "xpa_conv_dgrad_num_partials": (c_i64, [c_i64, c_i64, c_i64]),
    "xpa_conv_dgrad": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                      ctypes.c_int, c_p, c_f32, c_p, c_p, c_p]),
    "xpa_conv_wgrad_num_partials": (c_i64, []),
    "xpa_conv_wgrad_force_stream": (None, [ctypes.c_int]),
    "xpa_conv_wgrad": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_f32, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                      c_i64, c_p, c_p, c_p]),
    "xpa_rollout_bootstrap_fixup": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p]),
    "xpa_thin_bwd_num_partials": (c_i64, [c_i64]),
    "xpa_thin_linear_act_fwd_gather": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p,
                                                       c_f32, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "xpa_thin_linear_act_bwd_gather": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_p,
                                                       c_i64, c_i64, c_f32, c_p, c_p, c_p]),
    "xpa_thin_linear_act_fwd_norm": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f32,
                                                    c_p, c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_i64, c_p, c_p]),
    "xpa_thin_linear_act_fwd": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f32, c_p, c_i64,
                                               c_p]),
    "xpa_thin_linear_act_bwd": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_f32,
                                               c_p, c_p, c_p]),
    "xpa_head_gemm_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                                           c_p, c_i64, c_p, c_p, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_f32,
                                           c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32, c_p,
                                            c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_ws_grid": (c_i64, [c_i64]),
    "xpa_head_gemm_ws_probe": (ctypes.c_int, [ctypes.c_int]),
    "xpa_lds_poison": (ctypes.c_int, [c_p]),
    "xpa_head_gemm_ws_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                              c_p, c_p, c_i64, c_p, c_p, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                              c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_ws_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32,
                                               c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                              c_p, c_p, c_i64, c_p, c_p, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                              c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32,
                                               c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3p_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                              c_p, c_p, c_i64, c_p, c_p, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                              c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3p_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32,
                                               c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3q_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                              c_p, c_p, c_i64, c_p, c_p, c_f32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                              c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3q_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32,
                                               c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_trunk_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                                 c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32, c_p,
                                                 c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_f32, c_f32, c_p, c_p, c_p, c_p,
                                                 c_p, c_i64, c_p]),
    "xpa_head_gemm_trunk_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_f32, c_p,
                                                  c_i64, c_p, c_p, c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_f32, c_p,
                                                  c_p, c_p, c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3r_actor": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64, c_i64, c_i64, c_p, c_i64,
                                               c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p, c_p, c_i64, c_p, c_p, c_f32,
                                               c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_f32, c_f32, c_p, c_p, c_p,
                                               c_p, c_p, c_i64, c_p]),
    "xpa_head_gemm_s3r_critic": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_f32, c_p, c_p,
                                                c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p,
                                                c_i64, c_p]),
    "xpa_s3_gemm_trunk_bwd_sign": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, ctypes.c_int,
                                                  c_f32, c_p, c_p, c_p]),
    "xpa_thin_linear_act_fwd_gather_sign": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_p,
                                                           c_p, c_f32, c_p, c_i64, c_p, c_p, c_p, c_p, c_p]),
    "xpa_thin_probe": (ctypes.c_int, [ctypes.c_int]),
    "xpa_head_store_probe": (ctypes.c_int, [ctypes.c_int]),
    "xpa_head_stagger": (ctypes.c_int, [ctypes.c_int]),
    "xpa_s3_probe": (ctypes.c_int, [ctypes.c_int]),
    "xpa_head_gemm_s3q_critic_mask": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p,
                                                     c_f32, c_p, c_i64, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64, c_p,
                                                     c_p, c_p]),
    "xpa_s3_split_batch_scaled": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32,
                                                 c_p]),
    "xpa_s3_gemm_trunk_bwd_crit": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                                  c_i64, ctypes.c_int, c_f32, c_p, c_p, c_p]),
    "xpa_rollout_post_deferred_norm_rms": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_i64,
                                                          c_p, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p,
                                                          c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32, ctypes.c_int,
                                                          ctypes.c_int, c_f32, ctypes.c_int, c_p, c_p, c_p, c_i64, c_p,
                                                          c_p]),
    "xpa_s3_gemm_bias_act_rows": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, ctypes.c_int,
                                                 c_f32, c_p, c_p]),
    "xpa_s3_wgrad_rows": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "xpa_s3_gemm_rows_pair": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p]),
    "xpa_s3_split_batch_padded": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_s3_gemm_bias_act": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_p, ctypes.c_int, c_f32, c_p,
                                            c_p]),
    "xpa_s3_gemm_trunk_bwd_dz": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_p, c_i64, ctypes.c_int, c_f32, c_p, c_i64,
                                                c_p, c_p]),
    "xpa_s3_gemm_trunk_bwd_crit_dz": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                                     ctypes.c_int, c_f32, c_p, c_i64, c_p, c_p]),
    "xpa_gather_minibatch_pitched": (ctypes.c_int, [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "xpa_colsum_finalize_batch_map": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, ctypes.c_int,
                                                     ctypes.c_int, c_i64, c_i64, c_p, c_i64, c_f32, c_f32, c_p, c_p,
                                                     c_p]),
    "xpa_s3_wgrad_pair_slices": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p]),
    "xpa_s3_wgrad_pair_tune": (ctypes.c_int, [ctypes.c_int]),
    "xpa_s3_wgrad_pair": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_p, c_f32, c_i64, c_i64, c_i64,
                                         c_i64, c_p, c_p, c_p]),
    "xpa_s3_split_bytes": (c_i64, [c_i64, c_i64]),
    "xpa_s3_split_b": (ctypes.c_int, [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "xpa_s3_split_batch": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_p, c_p]),
    "xpa_s3_gemm": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "xpa_s3_gemm_group": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "xpa_s3_gemm_group_act_num_partials": (c_i64, [ctypes.c_int, c_i64]),
    "xpa_s3_gemm_group_act": (ctypes.c_int, [ctypes.c_int, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, ctypes.c_int,
                                             c_f32, c_i64, c_p, c_p]),
    "xpa_s3_wgrad_num_slices": (c_i64, [c_i64, c_i64]),
    "xpa_s3_gemm_trunk_bwd_num_partials": (c_i64, [c_i64]),
    "xpa_s3_gemm_trunk_bwd": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, ctypes.c_int,
                                             c_f32, c_p, c_p, c_p]),
    "xpa_s3_wgrad": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "xpa_s3_wgrad_padded": (ctypes.c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p]),
    "xpa_rollout_step_workspace": (c_i64, [c_i64, c_i64, ctypes.c_int, c_p]),
    "xpa_k14f_probe": (ctypes.c_int, [ctypes.c_int]),
    "xpa_s3_gemm_value": (ctypes.c_int, [c_p, c_i64, c_p, c_p, c_i64, c_i64, c_p, ctypes.c_int, c_f32, c_p, c_p, c_p]),
    "xpa_s3_gemm_rows_pair_trunk": (ctypes.c_int, [ctypes.c_int, c_p, c_i64, c_i64, c_p, c_p, c_f32, c_p, c_p, c_f32,
                                                   c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                                   c_p]),
    "xpa_rollout_step_synthbox": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f32,
                                                 c_p, c_p, c_p, c_p, c_p, c_p, c_u32, c_f32, c_p, c_p, c_p,
                                                 c_i64, c_p, c_u32, ctypes.c_int32, c_f32, c_f32, c_f32, c_p,
                                                 c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                                 c_p, c_p, c_i64, c_p, ctypes.c_int, c_p, c_p, c_p, c_f32, c_p, c_i64,
                                                 c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32, ctypes.c_int,
                                                 ctypes.c_int, c_f32, ctypes.c_int, c_p, c_p, c_p]),
    "xpa_grad_norm_num_partials": (c_i64, [c_i64]),
    "xpa_clip_adam_step": (ctypes.c_int, [c_p, c_p, c_p, c_p, c_i64, c_p, c_f32, c_f32, c_f32, c_f32, c_f32, c_i64, c_p,
                                          c_p]),
}

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall"]
OBJ_DIR = os.path.join(PKG_DIR, "_obj")

_lib = None


class XpaError(RuntimeError):
    pass


def _digest(paths, extra=""):
    import hashlib
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build_library(force=False, verbose=False, jobs=None):
    """Compile csrc/*.hip into libxuanpolicy_amd.so for gfx950 (cross-compiles without a GPU).

    One hipcc process per source file (in parallel, objects under xuanpolicy_amd/_obj/), then one link step.
    An object is rebuilt when the content hash of its source + the shared headers + the flags differs from the
    one recorded beside it (mtimes raced: a source edited while a build was running kept a stale object that
    looked newer than it)."""
    from concurrent.futures import ThreadPoolExecutor
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    headers = sorted([os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + [HEADER])
    hdr_digest = _digest(headers, " ".join(HIPCC_FLAGS))
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(OBJ_DIR, exist_ok=True)
    rebuilt = []

    def compile_one(src):
        obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
        want = _digest([src], hdr_digest)
        stamp = obj + ".sha256"
        if not force and os.path.exists(obj) and os.path.exists(stamp):
            with open(stamp) as f:
                if f.read().strip() == want:
                    return obj
        cmd = [hipcc] + HIPCC_FLAGS + ["-c", "-o", obj + ".tmp", src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        with open(stamp, "w") as f:
            f.write(want)
        rebuilt.append(obj)
        return obj
    jobs = jobs or min(len(srcs), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    link_stamp = LIB_PATH + ".sha256"
    link_want = _digest(objs)
    if not force and not rebuilt and os.path.exists(LIB_PATH) and os.path.exists(link_stamp):
        with open(link_stamp) as f:
            if f.read().strip() == link_want:
                return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    with open(link_stamp, "w") as f:
        f.write(link_want)
    return LIB_PATH


def load(path=None):
    """Load the library (once) and bind every exported symbol's signature."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise XpaError("libxuanpolicy_amd.so not built (%s); run __graft_entry__.build() or "
                       "xuanpolicy_amd._lib.build_library()" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.xpa_abi_version()
    if v != ABI_VERSION:
        raise XpaError("ABI version mismatch: library %d, bindings %d" % (v, ABI_VERSION))
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        raise XpaError("%s failed: hipError %d%s" % (what, rc, " (invalid argument)" if rc == 1 else ""))
