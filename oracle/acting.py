"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of the reference acting loop (`train_torch.py:171-358`):
`_pad_initial_state`, `_prepare_mcts_input`/`_encode_actions`, grayscale,
`_sample_action` (representation -> search), temperature sampling and recording
into per-env trajectories (`replay_buffer.py:ObservationTrajectory`), with injected
randomness: reset draws, Dirichlet noise (callback), ucb tie-breaks (keyed stream)
and action sampling by inverse CDF of u = uniform(env, STREAM_SAMPLE, step, 0)
(replaces `Categorical(probs).sample()` at train_torch.py:196-198).
"""
import numpy as np

from . import rng as R
from .env import BreakoutEnvOracle, convert_to_grayscale
from .mcts import MCTSOracle, NetModel
from . import nets as N

f32 = np.float32


def sample_probs(counts, temperature, vec_block=None, env_offset=0, n_envs_total=None, threads=1):
    """train_torch.py:192-193 bit for bit: `visit_counts ** (1/self.temperature)` on the whole (B, 3)
    int64 batch tensor (torch's CPU pow, restated in oracle/torch_pow.c: the element's position in the
    tensor decides between SLEEF's vector powf and the scalar double pow), then the f32 row sum
    ((c0 + c1) + c2, torch's order for a size-3 dim) and the f32 division."""
    from .torch_pow import pow_counts, VEC_BLOCK
    vt = pow_counts(counts, 1.0 / temperature, VEC_BLOCK if vec_block is None else vec_block, env_offset,
                    n_envs_total, threads)
    s = (vt[:, 0] + vt[:, 1]) + vt[:, 2]
    return (vt / s[:, None]).astype(np.float32)


def sample_actions(counts, temperature, u, vec_block=None, env_offset=0, n_envs_total=None, threads=1):
    """train_torch.py:192-198 with inverse-CDF sampling on injected u (f32) in place of
    `Categorical(probs[i]).sample()`. A shard passes its env_offset and the global env count."""
    probs = sample_probs(counts, temperature, vec_block, env_offset, n_envs_total, threads)
    B = counts.shape[0]
    out = np.zeros(B, dtype=np.int64)
    for b in range(B):
        cdf = f32(0)
        last = 0
        chosen = -1
        for a in range(3):
            if probs[b, a] > 0:
                last = a
            cdf = f32(cdf + probs[b, a])
            if chosen < 0 and u[b] < cdf:
                chosen = a
        out[b] = chosen if chosen >= 0 else last
    return out


class Trajectory:
    """ObservationTrajectory (replay_buffer.py:4-35) as plain lists."""

    def __init__(self, L, g0, pad_action=0):
        self.actions = [pad_action] * L
        self.states = [g0.copy() for _ in range(L - 1)]
        self.rewards = [0.0] * L
        self.visit_counts = [np.zeros(3, dtype=np.int64) for _ in range(L)]
        self.values = [0.0] * L
        self.length = 0
        self.reward_sum = 0.0

    def add_observation(self, action, state, reward, counts, value):
        self.actions.append(int(action))
        self.states.append(state.copy())
        self.rewards.append(f32(reward))
        self.visit_counts.append(counts.copy())
        self.values.append(f32(value))
        self.reward_sum = f32(self.reward_sum + f32(reward))
        self.length += 1


def prepare_mcts_input(cur_gray, traj, L, n_actions=3):
    """train_torch.py:259-293 -> (2L, H, W) f32."""
    acts = np.array(traj.actions[-L:], dtype=np.int64)
    planes = (acts.astype(np.float32) / f32(n_actions)).astype(np.float32)  # int64 tensor / int -> f32
    H, W = cur_gray.shape[-2:]
    aplanes = np.broadcast_to(planes[:, None, None], (L, H, W)).astype(np.float32)
    states = np.stack(traj.states[-(L - 1):]).reshape(-1, H, W)
    seq = np.concatenate([states, cur_gray.reshape(1, H, W)], axis=0)
    return np.concatenate([seq, aplanes], axis=0)


def run_episode(cfg, sd, seed, episode, noise_fn, n_parallel, max_steps=261, temperature=1.0,
                search_id0=0, step0=0, height=None, width=None, env_offset=0, on_step=None, n_envs_total=None):
    """One `_acting_stage` episode (train_torch.py:164-233) for `n_parallel` envs (a shard of
    `n_envs_total` starting at global env `env_offset`; default: the whole batch).

    Returns (trajectories, per-step log dict)."""
    mcfg = cfg["model"]
    L = mcfg["state_history_length"]
    env = BreakoutEnvOracle({**cfg["environment"], "n_parallel": n_parallel})
    if height:
        env.height = height
    if width:
        env.width = width
    state, _ = env.reset(env.reset_params(seed, episode, env_offset))
    g0 = convert_to_grayscale(state)
    trajs = [Trajectory(L, g0[b]) for b in range(n_parallel)]  # _pad_initial_state :313-332
    search = MCTSOracle(cfg, NetModel(sd, mcfg), seed)
    done = np.zeros(n_parallel, dtype=bool)
    prev_done = done  # train_torch.py:179 aliases the same object
    warp = convert_to_grayscale(state)
    t = 0
    log = []
    while not np.all(done):  # :184
        if t > max_steps - 1:  # :186 `length_counter > 260` with max_steps = 261
            break
        x = np.stack([prepare_mcts_input(warp[b], trajs[b], L) for b in range(n_parallel)])
        h = N.create_hidden_state_root(x, sd, mcfg)
        sid = search_id0 + t
        noise = noise_fn(sid, n_parallel)
        values, counts = search.search(h, noise, sid, env_offset)
        u = R.uniform(np.arange(n_parallel) + env_offset, R.STREAM_SAMPLE, step0 + t, 0, seed)
        action = sample_actions(counts, temperature, u, env_offset=env_offset, n_envs_total=n_envs_total)
        state, reward, done, valid = env.step(state, action, done)
        warp = convert_to_grayscale(state)
        rec = ~prev_done
        for b in range(n_parallel):
            if rec[b]:
                trajs[b].add_observation(action[b], warp[b], reward[b], counts[b], values[b])
        prev_done = done.copy()
        log.append({"action": action, "reward": reward, "done": done.copy(), "values": values,
                    "counts": counts, "valid": valid, "root_latent": h, "rep_input": x})
        if on_step is not None:
            on_step(t, log[-1])
        t += 1
    return trajs, log


def run_test_simulation(cfg, sd, seed, episode, noise_fn, batch=2, max_steps_test=200, temperature=0.1,
                        search_id0=0, step0=0, sd_rep=None):
    """RLSystem.run_test_simulation (train_torch.py:530-610) with injected randomness: padding
    action 1 (:545), temperature 0.1 sampling (:571-579), frames kept while the env is live
    (:583-585), and every env's trajectory extended every step with env 0's action (:594-598).
    The root latent comes from the learner net `sd_rep` (self.mu_zero, :567) and the search runs
    the target net `sd` (self.latent_mcts holds mu_zero_target, :91); sd_rep=None: the same net."""
    sd_rep = sd if sd_rep is None else sd_rep
    mcfg = cfg["model"]
    L = mcfg["state_history_length"]
    env = BreakoutEnvOracle({**cfg["environment"], "n_parallel": batch})
    state, _ = env.reset(env.reset_params(seed, episode))
    warp = convert_to_grayscale(state)
    trajs = [Trajectory(L, warp[b], pad_action=1) for b in range(batch)]
    search = MCTSOracle(cfg, NetModel(sd, mcfg), seed)
    done = np.zeros(batch, dtype=bool)
    frames = [[] for _ in range(batch)]
    step_i = 0
    while not np.all(done):
        if step_i > max_steps_test:
            break
        x = np.stack([prepare_mcts_input(warp[b], trajs[b], L) for b in range(batch)])
        h = N.create_hidden_state_root(x, sd_rep, mcfg)
        sid = search_id0 + step_i
        values, counts = search.search(h, noise_fn(sid, batch), sid, 0)
        u = R.uniform(np.arange(batch), R.STREAM_SAMPLE, step0 + step_i, 0, seed)
        action = sample_actions(counts, temperature, u)
        state, reward, done, valid = env.step(state, action, done)
        warp = convert_to_grayscale(state)
        for b in range(batch):
            if not done[b]:
                frames[b].append(warp[b].copy())
        step_i += 1
        for b in range(batch):
            trajs[b].add_observation(action[0], warp[b], reward[b], counts[b], values[b])
    return trajs, frames
