"""Precision envelopes of the production-net fixtures (test infrastructure; imports the oracle, never the reference).

A few Adam steps of an f32 network are chaotic in the last bits: Adam normalises every gradient element, so an
element whose f32 value is dominated by rounding (a near-zero sum, a max-pool argmax or ReLU kink decided by an ulp)
moves its weight by ~lr in a direction the rounding picks.  Two correct f32 implementations therefore drift apart
update by update (measured: the exact f64 replay of G9P leaves the f32 reference by 2.5e-7 in |TD| at update 0,
8e-6 at update 1, 7e-4 at update 2).  This script replays each fixture with the CPU oracle in float64 from the same
start and records, per checked quantity, how far the reference's own f32 result is from that exact replay.  The GPU
replay tests accept a deviation of max(base tolerance, 3 x this envelope): the device path must stay as close to the
reference as the reference itself is to exact arithmetic.

    python tests/golden/make_envelopes.py      (writes <fixture>_env.npz next to each fixture)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import cpu_ref  # noqa: E402
from oracle.synth_env import SynthAtariEnv  # noqa: E402
from tests.golden.fixture_init import uniform_state  # noqa: E402


def _load(name):
    return dict(np.load(os.path.join(HERE, name), allow_pickle=False))


def _perdqn_batch(seed, k, B, A):   # make_golden.perdqn_batch
    rng = np.random.default_rng(seed * 1000 + k)
    obs = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    nxt = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    act = rng.integers(0, A, B).astype(np.float32)
    rew = rng.normal(0, 1, B).astype(np.float32)
    term = (rng.random(B) < 0.2).astype(np.float32)
    return obs, act, rew, nxt, term


def envelope_perdqn(name="perdqn_prod.npz"):
    g = _load(name)
    B, A, n_up, seed, sync = (int(x) for x in g["config"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3
    pol = cpu_ref.build_qnetwork_ref(A, net[:nl], net[nl:2 * nl], net[2 * nl:3 * nl], net[3 * nl:])
    pol.load_state_dict({k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")})
    pol.double()
    opt = torch.optim.Adam(pol.parameters(), 1e-3, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.5, total_iters=10)
    lrn = cpu_ref.PerDQNLearnerRef(pol, opt, sch, float(g["gamma"]), sync)
    out = {"td": [], "info": []}
    for k in range(n_up):
        obs, act, rew, nxt, term = _perdqn_batch(seed, k, B, A)
        td, info = lrn.update(obs, act, rew, nxt, term)
        out["td"].append(np.abs(td - g["td_abs"][k]).max())
        out["info"].append(np.abs(np.asarray([info["Qloss"], info["learning_rate"], info["predictQ"]]) -
                                  g["infos"][k]))
    res = {"td": np.asarray(out["td"]), "info": np.stack(out["info"])}
    for key, v in pol.state_dict().items():
        res["sd/" + key] = np.asarray(np.abs(v.numpy() - g["sd%d/%s" % (n_up, key)]).max())
    np.savez_compressed(os.path.join(HERE, name.replace(".npz", "_env.npz")), **res)
    print(name, "td", res["td"], "info", res["info"].max(0))


def envelope_atari(name="atari_a2c_prod.npz"):
    g = _load(name)
    N, T, K, n_epoch, n_mb, max_ep, seed = (int(x) for x in g["config"])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3
    filters, kernels, strides, fc = net[:nl], net[nl:2 * nl], net[2 * nl:3 * nl], net[3 * nl:]
    pol = cpu_ref.build_atari_ac_ref(K, filters, kernels, strides, fc)
    small = "init_seed" not in g   # the small-net fixtures store their starting weights (sd0/)
    pre = "sd0/" if small else "sd0sum/"
    ref_keys = [k[len(pre):] for k in g if k.startswith(pre)]
    mine = list(pol.state_dict().keys())
    assert len(mine) == len(ref_keys)
    # the reference's state_dict order (representation, actor, critic) == the oracle's (critic_head last)
    order = [k for k in ref_keys if k.startswith("representation")] + [k for k in ref_keys if k.startswith("actor")] \
        + [k for k in ref_keys if k.startswith("critic")]
    shapes = [(k, pol.state_dict()[m].shape) for k, m in zip(order, mine)]
    vals = {k: g["sd0/" + k] for k, _ in shapes} if small else uniform_state(shapes, int(g["init_seed"]))
    pol.load_state_dict({m: torch.as_tensor(vals[k]) for k, m in zip(order, mine)})
    pol.double()
    ppo = int(g.get("algo", 0)) == 1   # G12P: PPOCLIP_Agent (ppo/atari.yaml coefficients, make_golden.capture_atari)
    if ppo:
        lr, vf, ent, clip, gn = (float(x) for x in g["hyper"])
    else:
        lr, vf, ent, clip, gn = 7e-4, 0.25, 0.01, 0.0, 0.2
    opt = torch.optim.Adam(pol.parameters(), lr, eps=1e-5)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=0.0, total_iters=10000)
    lrn = cpu_ref.LearnerRef(pol, opt, sch, "ppo" if ppo else "a2c", vf, ent, clip, gn, True)
    envs = [SynthAtariEnv(i, seed=seed, n_actions=K, max_episode_steps=max_ep) for i in range(N)]
    obs = np.stack([e.reset()[0] for e in envs])
    B = N * T // n_mb
    k = u = 0
    infos = []
    for it in range(g["act"].shape[0]):
        frames = np.zeros((N, T, 84, 84, 4), np.uint8)
        for t in range(T):
            acts = g["env_actions"][k]
            k += 1
            nxt, raw = obs.copy(), obs.copy()
            for i, e in enumerate(envs):
                o, r, te, tr, info = e.step(acts[i])
                if te or tr:
                    info["reset_obs"] = e.reset()[0]
                raw[i] = o
                nxt[i] = info["reset_obs"] if tr else o
            frames[:, t] = raw if (it, t) == (0, 0) else obs
            obs = nxt
        fl = frames.reshape(N * T, 84, 84, 4)
        act, ret, adv = g["act"][it].reshape(-1), g["ret"][it].reshape(-1), g["adv"][it].reshape(-1)
        for e in range(n_epoch):
            perm = g["perms"][it * n_epoch + e]
            for s in range(0, N * T, B):
                idx = perm[s:s + B]
                a = adv[idx]
                a = (a - a.mean()) / (a.std() + 1e-8)    # memory_tools.py:241-242 (sample's adv-norm)
                info = lrn.update(fl[idx], act[idx].astype(np.int64), ret[idx], a.astype(np.float32),
                                  old_logp=g["old_logp"][it].reshape(-1)[idx] if ppo else None)
                got = [info["actor-loss"], info["critic-loss"], info["entropy"], info["learning_rate"],
                       info["predict_value"]] + ([info["clip_ratio"]] if ppo else [])
                infos.append(np.abs(np.asarray(got) - g["infos"][u]))
                u += 1
    res = {"info": np.stack(infos)}
    sd = pol.state_dict()
    for key, m in zip(order, mine):
        a = sd[m].numpy()
        if "sd1/" + key in g:
            res["sd/" + key] = np.asarray(np.abs(a - g["sd1/" + key]).max())
        else:
            res["sd/" + key + "::rows16"] = np.asarray(np.abs(a[::16] - g["sd1/" + key + "::rows16"]).max())
            res["sd/" + key + "::rowsum"] = np.asarray(np.abs(a.reshape(a.shape[0], -1).sum(1) -
                                                              g["sd1/" + key + "::rowsum"]).max())
    np.savez_compressed(os.path.join(HERE, name.replace(".npz", "_env.npz")), **res)
    print(name, "info", res["info"].max(0), {k: float(v) for k, v in res.items() if k.startswith("sd/")})


if __name__ == "__main__":
    torch.set_num_threads(8)
    envelope_perdqn()
    envelope_atari()
    envelope_atari("atari_ppo_prod.npz")
    envelope_atari("atari_ppo.npz")
