"""ORACLE / TEST INFRASTRUCTURE — CPU (numpy) definition of the synthetic benchmark envs.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The GPU path (xuanpolicy_amd/csrc/rollout.hip: xpa_synthbox_step) implements the same math;
this file is the checker and the CPU baseline's environment.

The reference ships no synthetic env; BASELINE.md / SURVEY.md §8(d) define `SynthBox(D, A)` to be
plugged in through the reference's `NewEnv` hook (xuance/environment/__init__.py:76-78) with the
`New_Env` step contract (xuance/environment/new_env/new_env.py:27-42):
    reset() -> (obs, info{episode_step})
    step(a) -> (obs, reward, terminated, truncated, info{episode_step, episode_score})

Dynamics (all randomness from a stateless counter hash so CPU and GPU agree):
    x   = W s + U clip(a, -1, 1) + NOISE * xi          (Box actions)
    x   = W s + U[:, a] + NOISE * xi                     (Discrete actions)
    s'  = tanh(x);  r = -mean(s'^2);  terminated = s'[0] > TERM_THRESH
    truncated = episode_step >= max_episode_steps
    reset: s0 = 0.1 * (2u - 1)
    xi_d = sqrt(3) * (u1 + u2 + u3 + u4 - 2)   (mean 0, var 1),  u_j = hash_u01(seed, env, episode, (t*D+d)*4+j)
"""
import numpy as np

MASK32 = 0xFFFFFFFF
W_GAIN = 1.25
U_GAIN = 0.6
NOISE = 0.35
TERM_THRESH = 0.92
RESET_SCALE = 0.1
SALT_W = 0x57A7E000
SALT_U = 0x0AC7E000
SALT_RESET = 0x5EED0000


def mix32(x):
    """murmur3 fmix32 over a uint32 numpy array (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x85EBCA6B)
        x ^= x >> np.uint32(13)
        x *= np.uint32(0xC2B2AE35)
        x ^= x >> np.uint32(16)
    return x


def hash4(seed, k0, k1, k2):
    """h = mix(mix(mix(mix(seed) ^ k0) ^ k1) ^ k2), broadcasting uint32 keys."""
    s = mix32(np.uint32(seed & MASK32))
    h = mix32(s ^ np.asarray(k0, dtype=np.uint32))
    h = mix32(h ^ np.asarray(k1, dtype=np.uint32))
    h = mix32(h ^ np.asarray(k2, dtype=np.uint32))
    return h


def u01(h):
    """Top 24 bits of a uint32 hash -> float32 uniform in [0, 1) (exact on CPU and GPU)."""
    return (np.asarray(h, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def synthbox_params(seed, obs_dim, act_dim, discrete=False):
    """Dynamics matrices W [D, D] and U [D, A] (float32), drawn from the hash."""
    D, A = obs_dim, act_dim
    i = np.arange(D, dtype=np.uint32)[:, None]
    j = np.arange(D, dtype=np.uint32)[None, :]
    W = (2.0 * u01(hash4(seed, SALT_W, i, j)) - 1.0) * np.sqrt(3.0 / D) * W_GAIN
    ja = np.arange(A, dtype=np.uint32)[None, :]
    gain = U_GAIN if not discrete else 1.0
    U = (2.0 * u01(hash4(seed, SALT_U, i, ja)) - 1.0) * np.sqrt(3.0 / max(A if not discrete else 1, 1)) * gain
    return W.astype(np.float32), U.astype(np.float32)


def synthbox_noise(seed, env, episode, t, D):
    """xi [.., D] float32 for (env, episode, t) arrays of equal shape."""
    env = np.asarray(env, dtype=np.uint32)[..., None]
    ep = np.asarray(episode, dtype=np.uint32)[..., None]
    t = np.asarray(t, dtype=np.uint32)[..., None]
    d = np.arange(D, dtype=np.uint32)
    base = (t * np.uint32(D) + d) * np.uint32(4)
    acc = np.zeros(np.broadcast(env, d).shape, np.float32)
    for k in range(4):
        acc = acc + u01(hash4(seed, env, ep, base + np.uint32(k)))
    return (acc - np.float32(2.0)) * np.float32(np.sqrt(3.0))


def synthbox_reset_state(seed, env, episode, D):
    env = np.asarray(env, dtype=np.uint32)[..., None]
    ep = np.asarray(episode, dtype=np.uint32)[..., None]
    d = np.arange(D, dtype=np.uint32)
    return ((2.0 * u01(hash4(seed ^ SALT_RESET, env, ep, d)) - 1.0) * RESET_SCALE).astype(np.float32)


class _Box:
    def __init__(self, low, high, shape):
        self.low = np.full(shape, low, np.float32)
        self.high = np.full(shape, high, np.float32)
        self.shape = tuple(shape)
        self.dtype = np.float32


class _Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64


class SynthBoxEnv:
    """One environment instance (stepped one at a time, like the reference's DummyVecEnv_Gym,
    xuance/environment/gym/gym_vec_env.py:201-212)."""

    def __init__(self, obs_dim, act_dim, seed=1, env_index=0, discrete=False, max_episode_steps=1000,
                 spaces=None):
        self.D, self.A, self.seed, self.index = obs_dim, act_dim, seed, env_index
        self.discrete = discrete
        self.W, self.U = synthbox_params(seed, obs_dim, act_dim, discrete)
        self.max_episode_steps = max_episode_steps
        if spaces is not None:
            self.observation_space, self.action_space = spaces
        else:
            self.observation_space = _Box(-1.0, 1.0, (obs_dim,))
            self.action_space = _Discrete(act_dim) if discrete else _Box(-1.0, 1.0, (act_dim,))
        self.episode = -1
        self._episode_step = 0
        self._episode_score = 0.0
        self.state = None

    def close(self):
        pass

    def render(self, *a, **k):
        pass

    NOISE_CHUNK = 64  # NOISE * xi drawn for 64 steps at a time (same values, amortised hashing)

    def reset(self):
        self.episode += 1
        self._episode_step = 0
        self._episode_score = 0.0
        self._chunk_t0, self._chunk = -1, None
        self.state = synthbox_reset_state(self.seed, self.index, self.episode, self.D)
        return self.state.copy(), {"episode_step": 0}

    def _noise(self, t):
        # hash4(seed, env, ep, k) == mix32(prefix ^ k) with prefix = mix(mix(mix(seed) ^ env) ^ ep):
        # the prefix is fixed per episode, so a chunk costs one vectorised mix32 (same values).
        if self._chunk is None or not (0 <= t - self._chunk_t0 < self.NOISE_CHUNK):
            if self._chunk is None:
                self._prefix = mix32(mix32(mix32(np.uint32(self.seed & MASK32)) ^ np.uint32(self.index))
                                     ^ np.uint32(self.episode))
            k = (np.arange(t * self.D * 4, (t + self.NOISE_CHUNK) * self.D * 4, dtype=np.uint64)
                 & MASK32).astype(np.uint32)
            u = u01(mix32(self._prefix ^ k)).reshape(self.NOISE_CHUNK, self.D, 4)
            xi = (u[..., 0] + u[..., 1] + u[..., 2] + u[..., 3] - np.float32(2.0)) * np.float32(np.sqrt(3.0))
            self._chunk_t0 = t
            self._chunk = np.float32(NOISE) * xi
        return self._chunk[t - self._chunk_t0]

    def step(self, action):
        W, U = self.W, self.U
        if self.discrete:
            drive = U[:, int(action)]
        else:
            drive = U @ np.clip(np.asarray(action, np.float32), -1.0, 1.0)
        xi = self._noise(self._episode_step)
        s = np.tanh(W @ self.state + drive + xi)
        r = -float(s @ s) / self.D
        self._episode_step += 1
        self._episode_score += r
        term = bool(s[0] > TERM_THRESH)
        trunc = bool(self._episode_step >= self.max_episode_steps)
        self.state = s
        info = {"episode_step": self._episode_step, "episode_score": self._episode_score}
        return s.copy(), r, term, trunc, info


class DummyVecEnvRef:
    """DummyVecEnv_Gym / DummyVecEnv_Atari (xuance/environment/gym/gym_vec_env.py:148-231) restated over a list of
    env objects with the step contract above: the host VecEnv a reference user hands the agent.

      reset()      every env, rows saved into buf_obs (gym_vec_env.py:177-182)
      step(acts)   env e steps with acts[e]; a done env (terminated or truncated) is reset and its first observation
                   goes to infos[e]["reset_obs"]; buf_obs[e] = the step's observation (the final one of a done env)
                   is written IN PLACE; copies of buf_obs / rewards / flags / infos are returned (:201-212)

    buf_obs is one array for the object's life (float32, uint8 with atari=True), so an agent that keeps a reference
    to it across envs.step (ppoclip_agent.py:60 `obs = self.envs.buf_obs`) sees the step's writes — the reference's
    first-store alias.  record: every action array passed to step() is appended to .actions (the tests hand the
    device agent's draws to the oracle loop).

    rebind=True restates SubprocVecEnv_Gym's contract instead (gym_vec_env.py:89-121): reset() and step() bind a NEW
    buf_obs array (np.array of the workers' observations) rather than writing the old one, so an agent's reference
    taken before envs.step keeps the pre-step observations (no first-store alias), and a done env's reset_obs is
    np.array of the worker's one-element result tuple: shape (1,) + obs_shape."""

    def __init__(self, envs, observation_space=None, action_space=None, atari=False, rebind=False):
        self.rebind = bool(rebind)
        self.envs = list(envs)
        self.num_envs = len(self.envs)
        e0 = self.envs[0]
        self.observation_space = observation_space if observation_space is not None else e0.observation_space
        self.action_space = action_space if action_space is not None else e0.action_space
        self.obs_shape = tuple(self.observation_space.shape)
        self.buf_obs = np.zeros((self.num_envs,) + self.obs_shape, np.uint8 if atari else np.float32)
        self.buf_dones = np.zeros((self.num_envs,), bool)
        self.buf_trunctions = np.zeros((self.num_envs,), bool)
        self.buf_rews = np.zeros((self.num_envs,), np.float32)
        self.buf_infos = [{} for _ in range(self.num_envs)]
        self.max_episode_length = getattr(e0, "max_episode_steps", 1000)
        self.actions = []

    def reset(self):
        if self.rebind:
            res = [env.reset() for env in self.envs]
            self.buf_obs = np.array([o for o, _ in res])
            self.buf_infos = [i for _, i in res]
            return self.buf_obs.copy(), list(self.buf_infos)
        for e, env in enumerate(self.envs):
            obs, info = env.reset()
            self.buf_obs[e] = obs
            self.buf_infos[e] = info
        return self.buf_obs.copy(), list(self.buf_infos)

    def step(self, actions):
        self.actions.append(np.array(actions, copy=True))
        if self.rebind:
            res = [env.step(actions[e]) for e, env in enumerate(self.envs)]
            self.buf_obs = np.array([r[0] for r in res])
            self.buf_rews = np.array([r[1] for r in res])
            self.buf_dones = np.array([r[2] for r in res])
            self.buf_trunctions = np.array([r[3] for r in res])
            self.buf_infos = [r[4] for r in res]
            for e, env in enumerate(self.envs):
                if self.buf_dones[e] or self.buf_trunctions[e]:
                    self.buf_infos[e]["reset_obs"] = np.array((env.reset()[0],))
        else:
            for e, env in enumerate(self.envs):
                obs, self.buf_rews[e], self.buf_dones[e], self.buf_trunctions[e], self.buf_infos[e] = \
                    env.step(actions[e])
                if self.buf_dones[e] or self.buf_trunctions[e]:
                    self.buf_infos[e]["reset_obs"], _ = env.reset()
                self.buf_obs[e] = obs
        return (self.buf_obs.copy(), self.buf_rews.copy(), self.buf_dones.copy(), self.buf_trunctions.copy(),
                list(self.buf_infos))

    def close(self):
        pass


class SynthBoxVec:
    """numpy-vectorised variant of the same env ('second CPU variant with the env
    vectorised in numpy').  Same semantics as N SynthBoxEnv instances in a DummyVecEnv."""

    def __init__(self, n_envs, obs_dim, act_dim, seed=1, discrete=False, max_episode_steps=1000):
        self.N, self.D, self.A, self.seed = n_envs, obs_dim, act_dim, seed
        self.discrete = discrete
        self.W, self.U = synthbox_params(seed, obs_dim, act_dim, discrete)
        self.max_episode_steps = max_episode_steps
        self.env_ids = np.arange(n_envs, dtype=np.uint32)
        self.episode = np.zeros(n_envs, np.uint32)
        self.ep_step = np.zeros(n_envs, np.int64)
        self.ep_score = np.zeros(n_envs, np.float64)
        self.state = synthbox_reset_state(seed, self.env_ids, self.episode, obs_dim)
        self.num_envs = n_envs

    def reset(self):
        return self.state.copy()

    def step(self, actions):
        if self.discrete:
            drive = self.U.T[np.asarray(actions, np.int64)]
        else:
            drive = np.clip(np.asarray(actions, np.float32), -1.0, 1.0) @ self.U.T
        xi = synthbox_noise(self.seed, self.env_ids, self.episode, self.ep_step.astype(np.uint32), self.D)
        x = self.state @ self.W.T + drive + np.float32(NOISE) * xi
        s = np.tanh(x.astype(np.float32))
        r = -np.mean(s * s, axis=1).astype(np.float32)
        self.ep_step += 1
        self.ep_score += r
        term = s[:, 0] > TERM_THRESH
        trunc = self.ep_step >= self.max_episode_steps
        final = s.copy()
        done = term | trunc
        self.state = s
        if done.any():
            ids = np.nonzero(done)[0]
            self.episode[ids] += 1
            self.ep_step[ids] = 0
            self.ep_score[ids] = 0.0
            self.state[ids] = synthbox_reset_state(self.seed, self.env_ids[ids], self.episode[ids], self.D)
        return final, r, term, trunc, self.state.copy()


# ------------------------------------------------------------------------------------------------
# SynthAtari: the Atari-shaped synthetic env of SURVEY.md §8(d) (C3 / C5 shapes).
# Observation uint8 [84, 84, 4] (HWC frame stack, channel 3 = newest, as Atari_Env's LazyFrames
# concatenation, xuance/environment/gym/gym_env.py:212-241), Discrete(n_actions), reward in {-1, 0, 1}
# (np.sign, gym_env.py:230), lives with the reference's flag rules (gym_env.py:193-209):
#   life lost (lives > 0 left): terminated = True, truncated = False (the episode continues)
#   game over / step limit:     terminated = True, truncated = True  (reset)
# Dynamics (counter hash only):
#   dx(a) = ((a + 1) % 3 - 1) * 3;  px = clip(px + dx(a), 0, 76)                  (paddle column)
#   ball column bx(t) = hash4(seed ^ SALT_BALL, env, ep, t >> 4) % 77, row by(t) = (t & 15) * 5
#   at t & 15 == 15: r = +1 if |px - bx(t)| <= 8 else -1 (a life lost); else r = 0
#   frame(ep, t, px)[y, x] = hash4(seed ^ SALT_PIX, env, ep, y*84 + x) >> 27    (static noise 0..31)
#                            255 inside the 8x8 ball at (by(t), bx(t)), 200 on the paddle rows 78..81
#   step: t = ep_step; ... ep_step += 1; new frame(ep, ep_step, px) pushed onto the stack
#   reset: lives 5, px 38, ep_step 0, stack = 4 copies of frame(ep, 0, 38)
# ------------------------------------------------------------------------------------------------
ATARI_HW = 84
ATARI_STACK = 4
ATARI_LIVES = 5
ATARI_PX0 = 38
SALT_PIX = 0xA7A21000
SALT_BALL = 0xBA11B000


def atari_dx(a):
    return ((np.asarray(a, np.int64) + 1) % 3 - 1) * 3


def atari_ball(seed, env, ep, t):
    bx = hash4(seed ^ SALT_BALL, env, ep, np.uint32(int(t) >> 4)) % np.uint32(77)
    return int(bx), (int(t) & 15) * 5


def atari_frame(seed, env, ep, t, px):
    p = np.arange(ATARI_HW * ATARI_HW, dtype=np.uint32)
    f = (hash4(seed ^ SALT_PIX, env, ep, p) >> np.uint32(27)).astype(np.uint8).reshape(ATARI_HW, ATARI_HW)
    bx, by = atari_ball(seed, env, ep, t)
    f[by:by + 8, bx:bx + 8] = 255
    f[78:82, px:px + 8] = 200
    return f


class SynthAtariEnv:
    """One SynthAtari env with the Atari_Env step contract (obs, reward, terminated, truncated, info)."""

    def __init__(self, env_id, seed=1, n_actions=6, max_episode_steps=27000):
        self.env_id, self.seed, self.n_actions, self.max_episode_steps = int(env_id), int(seed), n_actions, max_episode_steps
        self.ep = 0
        self._reset_state()

    def _reset_state(self):
        self.lives, self.px, self.ep_step, self.score = ATARI_LIVES, ATARI_PX0, 0, 0.0
        f = atari_frame(self.seed, self.env_id, self.ep, 0, self.px)
        self.stack = np.repeat(f[:, :, None], ATARI_STACK, axis=2)

    def reset(self):
        return self.stack.copy(), {"episode_step": 0}

    def step(self, a):
        t = self.ep_step
        self.px = int(np.clip(self.px + int(atari_dx(a)), 0, 76))
        r = 0.0
        if (t & 15) == 15:
            bx, _ = atari_ball(self.seed, self.env_id, self.ep, t)
            r = 1.0 if abs(self.px - bx) <= 8 else -1.0
        self.ep_step += 1
        self.score += r
        if r < 0:
            self.lives -= 1
        game_over = self.lives == 0 or self.ep_step >= self.max_episode_steps
        terminated = bool(game_over or r < 0)
        truncated = bool(game_over)
        f = atari_frame(self.seed, self.env_id, self.ep, self.ep_step, self.px)
        self.stack = np.concatenate([self.stack[:, :, 1:], f[:, :, None]], axis=2)
        obs = self.stack.copy()
        info = {"episode_step": self.ep_step, "episode_score": self.score}
        if game_over:
            self.ep += 1
            self._reset_state()
            info["reset_obs"] = self.stack.copy()
        return obs, np.float32(r), terminated, truncated, info


# ---------------------------------------------------------------------------------------------------------------
# CartPole-v1 (BASELINE.json configs[0]).  gym is not installed here; this restates the published
# gym 0.26.2 classic_control/cartpole.py dynamics (euler integrator, Python-float = f64 state, f32 observations)
# under TimeLimit(max_episode_steps=500).  Delta: the reset state's uniform(-0.05, 0.05) draws come from the
# counter hash (seed, env, episode, dim) instead of the env's np_random, so CPU and GPU agree.  Parity against
# gym itself is unpinned (no gym, no recorded gym trajectories in the reference).
CP_GRAVITY, CP_MASSCART, CP_MASSPOLE, CP_LENGTH, CP_FORCE, CP_TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
CP_TOTAL_MASS = CP_MASSPOLE + CP_MASSCART
CP_POLEMASS_LENGTH = CP_MASSPOLE * CP_LENGTH
CP_THETA_THRESHOLD = 12 * 2 * np.pi / 360
CP_X_THRESHOLD = 2.4
SALT_CARTPOLE = 0xCA27B01E


def cartpole_reset_state(seed, env, episode):
    """uniform(-0.05, 0.05) per dim: f32-exact hash uniform, then f64 (the device computes the same)."""
    u = u01(hash4(seed ^ SALT_CARTPOLE, np.uint32(env), np.uint32(episode), np.arange(4, dtype=np.uint32)))
    return u.astype(np.float64) * 0.1 - 0.05


def cartpole_dynamics(state, action):
    """One euler step of gym's CartPoleEnv.step (cartpole.py: force, temp, thetaacc, xacc, euler update) on f64
    state arrays [..., 4]; returns (new_state, terminated)."""
    x, x_dot, theta, theta_dot = (state[..., k] for k in range(4))
    force = np.where(np.asarray(action) == 1, CP_FORCE, -CP_FORCE)
    costheta, sintheta = np.cos(theta), np.sin(theta)
    temp = (force + CP_POLEMASS_LENGTH * theta_dot ** 2 * sintheta) / CP_TOTAL_MASS
    thetaacc = (CP_GRAVITY * sintheta - costheta * temp) / (
        CP_LENGTH * (4.0 / 3.0 - CP_MASSPOLE * costheta ** 2 / CP_TOTAL_MASS))
    xacc = temp - CP_POLEMASS_LENGTH * thetaacc * costheta / CP_TOTAL_MASS
    x = x + CP_TAU * x_dot
    x_dot = x_dot + CP_TAU * xacc
    theta = theta + CP_TAU * theta_dot
    theta_dot = theta_dot + CP_TAU * thetaacc
    new = np.stack([x, x_dot, theta, theta_dot], axis=-1)
    term = (x < -CP_X_THRESHOLD) | (x > CP_X_THRESHOLD) | (theta < -CP_THETA_THRESHOLD) | (theta > CP_THETA_THRESHOLD)
    return new, term


class CartPoleEnv:
    """One CartPole-v1 env with the gym step contract the reference's DummyVecEnv_Gym drives (reward 1 per step,
    terminated on the angle / position limits, truncated at 500 steps, auto-reset by the vec env)."""

    def __init__(self, env_id, seed=1, max_episode_steps=500):
        self.env_id, self.seed, self.max_episode_steps = int(env_id), int(seed), int(max_episode_steps)
        self.ep = 0
        self.D, self.A, self.discrete = 4, 2, True   # AgentLoopRef's env description
        self.observation_space = _Box(-np.inf, np.inf, (4,))
        self.action_space = _Discrete(2)
        self._reset_state()

    def _reset_state(self):
        self.state = cartpole_reset_state(self.seed, self.env_id, self.ep)
        self.ep_step, self.score = 0, 0.0

    def reset(self):
        return self.state.astype(np.float32), {"episode_step": self.ep_step}

    def close(self):
        pass

    def step(self, a):
        self.state, term = cartpole_dynamics(self.state, int(a))
        self.ep_step += 1
        self.score += 1.0
        term = bool(term)
        trunc = self.ep_step >= self.max_episode_steps   # gym TimeLimit: independent of terminated
        obs = self.state.astype(np.float32)
        info = {"episode_step": self.ep_step, "episode_score": self.score}
        if term or trunc:
            self.ep += 1
            self._reset_state()
        return obs, np.float32(1.0), term, trunc, info
