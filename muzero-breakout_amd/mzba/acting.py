"""Fused on-device acting loop (mirror of train_torch.py:160-233 `_acting_stage` /
`_run_episode` / `_sample_action`).

One acting step = rep-input assembly from the frame-history ring (:259-293) ->
representation + min-max scaling (:254) -> latent MCTS (:256) -> temperature
sampling (:191-198) -> env step + gray render + history push + trajectory record
(:201-209). Everything stays on the device; the per-step records land in a device
trajectory sink (replay_buffer.py:ObservationTrajectory fields) that is copied to the
host once per episode (or gathered to rank 0 over RCCL for multi-GPU runs).
"""
import numpy as np
import torch

from . import _lib as L
from .env import CompactBreakout, gray_lut
from .search import MCTSSearchVec, SearchWorkspace


class ObservationTrajectory:
    """Host record with the reference's fields (replay_buffer.py:4-35)."""

    def __init__(self, actions, states, rewards, visit_counts, values, length, reward_sum):
        self.actions, self.states, self.rewards = actions, states, rewards
        self.visit_counts, self.values = visit_counts, values
        self.length, self.reward_sum = length, reward_sum

    def add_observation(self, action, state, reward, visit_counts, values):
        self.actions.append(action); self.states.append(state); self.rewards.append(reward)
        self.visit_counts.append(visit_counts); self.values.append(values)
        self.reward_sum += reward
        self.length += 1

    def get_actions(self):
        return torch.tensor(self.actions)

    def get_states(self):
        return torch.stack(self.states)

    def get_rewards(self):
        return torch.tensor(self.rewards)

    def get_visit_counts(self):
        return torch.stack(self.visit_counts)

    def get_values(self):
        return torch.tensor(self.values)

    def get_reward_sum(self):
        return self.reward_sum


class ActingLoop:
    """B envs acting with MCTS on one device. `env_offset` = global id of env 0 (sharding)."""

    MAX_STEPS = 261  # train_torch.py:186 `length_counter > 260`

    # torch's CPU pow takes 2 x Vectorized<float>::size() elements per vector iteration; 32 on the
    # AVX512 host the reference fixtures were generated on (16 on an AVX2 host), csrc/torch_pow.h
    VEC_BLOCK = 32

    def __init__(self, cfg, agent, B, seed=0, env_offset=0, temperature=1.0, height=16, width=20,
                 record_frames=True, max_steps=MAX_STEPS, pad_action=0, rec_flags=0, n_envs_total=None,
                 rep_agent=None, pow_threads=None):
        """`n_envs_total`: envs of the whole (sharded) batch, the reference's visit_counts tensor
        (default env_offset + B); `rep_agent`: the net of the root representation when it differs
        from the search's (run_test_simulation: learner net for the root, target net in the search);
        `pow_threads`: intra-op threads of the reference's torch process, which split its visit-count
        pow into per-thread chunks from 32768 elements on (3 x n_envs_total >= 32768); default
        cfg["pow_threads"], else 1."""
        self.cfg, self.agent, self.B = cfg, agent, B
        self.seed, self.env_offset = seed, env_offset
        self.n_envs_total = env_offset + B if n_envs_total is None else n_envs_total
        self.max_steps = max_steps
        # the reference process's intra-op thread count is a property of ITS launch, not of this one:
        # explicit (argument, else cfg["pow_threads"], else 1 — what the oracle assumes), never inferred
        self.pow_threads = int(cfg.get("pow_threads", 1) if pow_threads is None else pow_threads)
        dev = agent.device
        # graph-replayable schedule values (train_torch.py:129-135): 1/T in double for the sampling
        # kernel, (f32(1 - noise_weight), f32(noise_weight)) for the root expansion
        self.inv_t_dev = torch.ones(1, dtype=torch.float64, device=dev)
        self.root_w_dev = torch.zeros(2, dtype=torch.float32, device=dev)
        self._temperature = None
        self._noise_weight = None
        self.temperature = temperature
        mcfg = cfg["model"]
        self.Lh = mcfg["state_history_length"]
        self.H, self.W = height, width
        dev = agent.device
        self.env = CompactBreakout(cfg["environment"], B, self.Lh, height, width, seed=seed, env_offset=env_offset,
                                   device=dev, pad_action=pad_action, rec_flags=rec_flags)
        self.search = MCTSSearchVec(cfg, agent, None, seed=seed, env_offset=env_offset)
        self.ws = SearchWorkspace(self.search, B)
        p = agent.packed
        self.cs = (2 * self.Lh + 63) // 64 * 64
        self.rep_in = torch.empty(B * height * width * self.cs, dtype=p.tdt, device=dev)
        self.rep_agent = agent if rep_agent is None else rep_agent
        if self.rep_agent.packed.tdt != p.tdt or self.rep_agent.device != dev:
            raise ValueError("rep_agent must share the search agent's device and dtype")
        self.rep_runner = self.rep_agent.runner(B, height, width)
        self.action = torch.zeros(B, dtype=torch.int64, device=dev)
        T = max_steps
        self.rec = {
            "action": torch.zeros(T, B, dtype=torch.uint8, device=dev),
            "reward": torch.zeros(T, B, dtype=torch.float32, device=dev),
            "mask": torch.zeros(T, B, dtype=torch.uint8, device=dev),
            "frame": torch.zeros(T, B, height * width, dtype=torch.uint8, device=dev) if record_frames else None,
            "counts": torch.zeros(T, B, 3, dtype=torch.int64, device=dev),
            "values": torch.zeros(T, B, dtype=torch.float32, device=dev),
        }
        self.noise_log = None  # optional list: per-step Dirichlet noise used (parity tests)
        # optional callable (search_id, B) -> f32 (B, 3): root Dirichlet noise injected in place of the
        # device draw (replaying the reference's fixtures, whose noise came from their own generator);
        # steps then run eagerly
        self.inject_noise = None
        self._noise_in = None
        self.search_id = 0
        self.step_index = 0
        self.episode = 0
        # device step context [search id, step index, episode row t]: every per-step varying
        # value is read from here, so one captured HIP graph replays every acting step
        self.ctx = torch.zeros(3, dtype=torch.int32, device=dev)
        self.graph = None

    @property
    def temperature(self):
        return self._temperature

    @temperature.setter
    def temperature(self, t):
        """train_torch.py:129-132; the captured step graph reads 1/T from inv_t_dev."""
        if t != self._temperature:
            self._temperature = t
            self.inv_t_dev.fill_(1.0 / t)  # Python's `1/self.temperature` (double), train_torch.py:192

    def _sync_noise_weight(self):
        w = self.search.noise_weight  # train_torch.py:134-135 sets it on the search object
        if w != self._noise_weight:
            self._noise_weight = w
            self.root_w_dev.copy_(torch.tensor([np.float32(1 - w), np.float32(w)], dtype=torch.float32))

    def reset(self, episode=None, params=None):
        """_acting_stage :166-167: env.reset + _pad_initial_state."""
        if episode is not None:
            self.episode = episode
        self.env.reset(self.episode, params)
        self.frame0 = self.env.current_frame()
        self.episode += 1
        self.t = 0
        self.ctx.copy_(torch.tensor([self.search_id, self.step_index, 0], dtype=torch.int32))

    def _act_body(self):
        """One acting step, every launch stream-ordered and parameterised by self.ctx."""
        env, ws = self.env, self.ws
        n = ws.n
        # _prepare_mcts_input + create_hidden_state_root -> pool slot 0
        env.build_rep_input(self.rep_in, self.cs, self.agent.dtype == "bf16")
        self.rep_runner.representation(self.rep_in, ws.cur, pool=ws.pool, pool_env_stride=(ws.S + 1) * n)
        values, counts = ws.run(self.search_id, self._noise_in, ctx=self.ctx, w_dev=self.root_w_dev)
        L.call("mzba_sample_actions", L.ptr(counts), L.ptr(self.action), None, self.B, 1.0 / self.temperature,
               L.ptr(self.inv_t_dev), self.n_envs_total, self.VEC_BLOCK, self.pow_threads, self.env_offset,
               self.step_index, self.seed,
               L.ptr(self.ctx), L.stream())
        L.call("mzba_record_results", L.ptr(counts), L.ptr(values), L.ptr(self.rec["counts"]),
               L.ptr(self.rec["values"]), self.B, 0, L.ptr(self.ctx), L.stream())
        env.step(self.action, False, self.rec, 0, ctx=self.ctx)
        L.call("mzba_ctx_advance", L.ptr(self.ctx), L.stream())

    def capture(self):
        """Capture one acting step (~S x 65 launches) into a HIP graph; act() then replays it.
        Temperature and noise weight are read from device buffers, so the graph stays valid across
        the reference's schedule. The captured step draws its root noise on the device."""
        if self.inject_noise is not None:
            raise RuntimeError("capture(): injected noise is host data per step; clear inject_noise first")
        self._noise_in = None
        self._sync_noise_weight()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._act_body()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = g

    def act(self, eager=False):
        """One acting step t (no host synchronisation)."""
        self._sync_noise_weight()
        if self.inject_noise is not None:
            nz = np.ascontiguousarray(self.inject_noise(self.search_id, self.B), dtype=np.float32)
            self._noise_in = torch.from_numpy(nz).to(self.agent.device)
            eager = True
        else:  # back to the device Dirichlet draw (a later capture must not bake in the last injected rows)
            self._noise_in = None
        if self.graph is not None and not eager and self.noise_log is None:
            self.graph.replay()
        else:
            self._act_body()
            if self.noise_log is not None:
                self.noise_log.append(self.ws.tree.noise.clone())
        self.search_id += 1
        self.step_index += 1
        self.t += 1

    def all_done(self):
        return bool(self.env.done.bool().all().item())

    def run_episode(self, episode=None, params=None):
        """_run_episode :171-233 -> list of ObservationTrajectory (host)."""
        self.reset(episode, params)
        while not self.all_done():
            if self.t >= self.max_steps:
                break
            self.act()
        return self.trajectories()

    def trajectories(self):
        """Per-env ObservationTrajectory exactly as _pad_initial_state + add_observation
        build them (31 padding frames of g(s0), 32 padding actions 0, then the records)."""
        return trajectories_from_records(self.rec, self.frame0, self.t, self.Lh, self.H, self.W, self.env.pad_action)


def trajectories_from_records(rec, frame0, T, L_, H, W, pad_action=0):
    """The sink's first T rows (dict of (T_max, B, ...) tensors) + the u8 g(s0) codes (B*H*W) ->
    one ObservationTrajectory per env, as _pad_initial_state (train_torch.py:313-332) and the
    recording loop (:204-209) build them."""
    rec = {k: (v[:T].cpu().numpy() if v is not None else None) for k, v in rec.items()}
    B = rec["action"].shape[1]
    lut = gray_lut()
    f0 = frame0.reshape(B, H * W).cpu().numpy()
    out = []
    for b in range(B):
        m = rec["mask"][:, b].astype(bool)
        acts = [pad_action] * L_ + [int(a) for a in rec["action"][m, b]]
        pad = torch.from_numpy(lut[f0[b] & 7].reshape(1, H, W))
        states = [pad] * (L_ - 1)
        if rec.get("frame") is not None:
            states += [torch.from_numpy(lut[f & 7].reshape(1, H, W)) for f in rec["frame"][m, b]]
        rews = [0] * L_ + [float(r) for r in rec["reward"][m, b]]
        vc = [torch.zeros(3)] * L_ + [torch.from_numpy(c) for c in rec["counts"][m, b]]
        vals = [0.0] * L_ + [float(v) for v in rec["values"][m, b]]
        rs = np.float32(0)
        for r in rec["reward"][m, b]:
            rs = np.float32(rs + r)
        out.append(ObservationTrajectory(acts, states, rews, vc, vals, int(m.sum()), float(rs)))
    return out


def run_test_simulation(cfg, agent, batch=2, seed=0, episode=0, max_steps_test=200, temperature=0.1,
                        log_noise=False, rep_agent=None):
    """RLSystem.run_test_simulation (train_torch.py:530-610) on the device: `batch` envs played
    at temperature 0.1 until all are done or after max_steps_test + 1 steps, with the reference's
    quirks (padding action 1, every env recorded every step with env 0's action). `agent` is the
    search's net (self.latent_mcts holds the target net, train_torch.py:91) and `rep_agent` the
    root representation's (self.mu_zero, the learner net, :567; default: `agent`). Returns
    (ObservationTrajectory per env, frames per env: the grayscale (1, H, W) frames of the steps
    after which the env was still live — what the reference logs — and the loop). The reference
    writes the frames of env 0 to tensorboard; logging is left to the caller."""
    loop = ActingLoop(cfg, agent, batch, seed=seed, temperature=temperature, max_steps=max_steps_test + 1,
                      pad_action=1, rec_flags=3, rep_agent=rep_agent)
    loop.noise_log = [] if log_noise else None
    loop.reset(episode)
    H, W = loop.H, loop.W
    lut = gray_lut()
    frames = [[] for _ in range(batch)]
    step_i = 0
    while not loop.all_done():  # :559
        if step_i > max_steps_test:  # :562
            break
        loop.act(eager=True)
        done = loop.env.done.cpu().numpy().astype(bool)
        cur = loop.env.current_frame().view(batch, -1).cpu().numpy()
        for b in range(batch):  # :583-585
            if not done[b]:
                frames[b].append(torch.from_numpy(lut[cur[b] & 7].reshape(1, H, W)))
        step_i += 1
    return loop.trajectories(), frames, loop


class ActingStage:
    """Mirror of RLSystem._acting_stage (train_torch.py:160-169): `num_episodes` episodes of the
    `n_parallel` envs of cfg with the target agent, each run until every env is done or after 261 steps
    (:184-187), the records going where the reference sends them (:222-225).

    Sharded: with `world_size` > 1 (one process per GPU, torch.distributed initialised —
    backend "nccl" = RCCL over xGMI) rank r runs the global envs [r*B, (r+1)*B), B = n_parallel /
    world_size, every random draw keyed on the global env id and the temperature pow on the envs'
    global positions (n_envs_total = n_parallel); the ranks step in lockstep until the whole global batch
    is done (one all-reduce of a live flag per step), and every `record_k` steps their record rows are
    gathered to rank 0 (`mzba.shard.ShardedSink`). Rank 0 then holds the episode as one loop over the
    global batch would have recorded it, bit for bit, and saves it into `replay_buffer`
    (`DeviceReplayBuffer.ingest_records`: windows + n-step targets of every trajectory longer than K + 1,
    in global env order) and/or returns the per-env ObservationTrajectory lists.
    `temperature` / `noise_weight` follow the caller's schedule (train_torch.py:129-135)."""

    def __init__(self, cfg, agent, seed=0, env_offset=0, use_graph=True, world_size=1, rank=0, record_k=16,
                 pow_threads=None, max_steps=ActingLoop.MAX_STEPS, height=16, width=20):
        n = cfg["n_parallel"]
        if world_size < 1 or not 0 <= rank < world_size or n % world_size:
            raise ValueError(f"ActingStage: n_parallel {n} must split evenly over world_size {world_size}")
        self.cfg = cfg
        self.world, self.rank = world_size, rank
        B = n // world_size
        self.loop = ActingLoop(cfg, agent, B, seed=seed, env_offset=env_offset + rank * B,
                               n_envs_total=env_offset + n, pow_threads=pow_threads, max_steps=max_steps,
                               height=height, width=width)
        self.use_graph = use_graph
        self.num_episodes = cfg["num_episodes"]
        self.sink = None
        if world_size > 1:
            from .shard import ShardedSink
            self.sink = ShardedSink(world_size, rank, record_k, B, height * width, max_steps, agent.device)

    @property
    def temperature(self):
        return self.loop.temperature

    @temperature.setter
    def temperature(self, t):
        self.loop.temperature = t  # a device value: the captured step graph stays valid

    def set_noise_weight(self, w):
        self.loop.search.noise_weight = w  # copied to the device before the next step

    def _all_done(self):
        if self.sink is None:
            return self.loop.all_done()
        from .shard import all_ranks_done
        return all_ranks_done(self.loop.env.done)

    def run_episode(self, replay_buffer=None, trajectories=True):
        """One episode (_acting_stage :166-167 + _run_episode :171-233). Returns the per-env
        ObservationTrajectory list of the global batch on rank 0 (None elsewhere, or when not
        `trajectories`); rank 0 saves the episode into `replay_buffer` when one is given."""
        loop, sink = self.loop, self.sink
        if sink is not None:
            sink.gather.fence()
        loop.reset()
        if sink is not None:
            sink.begin(loop.frame0)
        while not self._all_done() and loop.t < loop.max_steps:
            loop.act()
            if self.use_graph and loop.graph is None:
                loop.capture()
            if sink is not None:
                sink.push(loop.rec, loop.t)
        if sink is not None:
            rec, frame0 = sink.finish(loop.rec, loop.t)
        else:
            rec, frame0 = loop.rec, loop.frame0
        if self.rank != 0:
            return None
        if replay_buffer is not None:
            replay_buffer.ingest_records(rec, frame0.reshape(-1, loop.H * loop.W), loop.t)
        if trajectories:
            return trajectories_from_records(rec, frame0, loop.t, loop.Lh, loop.H, loop.W, loop.env.pad_action)
        return None

    def run(self, replay_buffer=None, trajectories=True):
        """`num_episodes` episodes -> a list of run_episode results."""
        return [self.run_episode(replay_buffer, trajectories) for _ in range(self.num_episodes)]
