"""Generate the golden fixtures in tests/golden/*.npz FROM THE REFERENCE ITSELF.

Runs only in the build container (needs /root/reference); the committed .npz files
are data (inputs + expected outputs). The reference is imported through
ref_harness (stubs + device remap, nothing edited) and its torch RNG calls are
replaced by draws from the keyed Philox stream (oracle/rng.py) so the oracle and
the HIP kernels can consume identical randomness:
  parallel_breakout.py torch.randint -> randbelow(env, STREAM_RESET, episode, kind)
  mcts.py Dirichlet(...).sample()     -> injected noise rows (stored in fixture)
  mcts.py torch.randint(len(best))    -> randbelow(env, STREAM_TIE, search_id, k)
  train_torch.py Categorical.sample() -> inverse CDF of uniform(env, STREAM_SAMPLE, t, 0)

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))

import ref_harness  # noqa: E402

ref_harness.install()
import torch  # noqa: E402

from oracle import rng as R  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402

SEED = 20251015
torch.set_num_threads(8)


class Proxy:
    """Module proxy: attribute overrides, everything else forwarded to `base`."""

    def __init__(self, base, **over):
        self._base, self._over = base, over

    def __getattr__(self, name):
        if name in self._over:
            return self._over[name]
        return getattr(self._base, name)


# --------------------------------------------------------------------------------------
# env reset injection
class ResetInjector:
    def __init__(self, seed):
        self.seed, self.episode, self.calls, self.batch = seed, 0, 0, None

    def begin(self, batch):
        self.calls, self.batch = 0, batch

    def randint(self, *args, **kwargs):
        if len(args) == 3:
            low, high, size = args
        elif len(args) == 2 and isinstance(args[1], tuple):
            low, (high, size) = 0, args
        else:
            low, high, size = args[0], args[1], kwargs.get("size")
        c = self.calls
        self.calls += 1
        if c < 3:
            env = np.arange(self.batch)
            kind = c
        else:
            env = np.array([c - 3])
            kind = 3
        v = low + R.randbelow(env, R.STREAM_RESET, self.episode, kind, self.seed, high - low)
        return torch.from_numpy(v.astype(np.int64))


def patched_env_class(inj):
    import environment.parallel_breakout as pb

    pb.torch = Proxy(torch, randint=inj.randint)
    Base = pb.BreakoutEnvironment

    class Env(Base):
        def reset(self):
            inj.begin(self.batch)
            out = super().reset()
            inj.episode += 1
            return out

    return Env


def pack_state(s):
    """(B,3,H,W) {0,1} f32 -> bit-packed uint8 (B,3,ceil(H*W/8))."""
    a = np.asarray(s)
    assert np.all((a == 0) | (a == 1))
    B = a.shape[0]
    return np.packbits(a.reshape(B, 3, -1).astype(np.uint8), axis=-1)


# --------------------------------------------------------------------------------------
def make_env(cfg):
    out = {}
    inj = ResetInjector(SEED)
    Env = patched_env_class(inj)
    for tag, (B, H, W, T) in {"16x20": (32, None, None, 261), "84x84": (8, 84, 84, 300)}.items():
        e = Env({**cfg["environment"], "n_parallel": B})
        if H:
            e.height, e.width = H, W
        inj.episode = 0
        state, _ = e.reset()
        done = torch.zeros(B, dtype=torch.bool)
        states, rewards, dones, valids, dxs, dys, acts = [pack_state(state)], [], [], [], [], [], []
        dxs.append(e.ball_dx.numpy().copy()); dys.append(e.ball_dy.numpy().copy())
        for t in range(T):
            a = R.randbelow(np.arange(B), 7, t, 0, SEED, 3)  # fixture-only action stream
            act = torch.from_numpy(a)
            state, r, done, v = e.step(state, act, done)
            acts.append(a); states.append(pack_state(state)); rewards.append(r.numpy().copy())
            dones.append(done.numpy().copy()); valids.append(v.numpy().copy())
            dxs.append(e.ball_dx.numpy().copy()); dys.append(e.ball_dy.numpy().copy())
        out[tag] = dict(B=B, H=H or 16, W=W or 20, actions=np.stack(acts), states=np.stack(states),
                        rewards=np.stack(rewards), dones=np.stack(dones), valids=np.stack(valids),
                        dx=np.stack(dxs), dy=np.stack(dys))
    for tag, d in out.items():
        np.savez_compressed(os.path.join(HERE, f"env_{tag}.npz"), seed=SEED, **d)
        print("env", tag, {k: getattr(v, "shape", v) for k, v in d.items()},
              "reward set", np.unique(d["rewards"]), "done frac", d["dones"][-1].mean())


def make_env_fuzz(cfg):
    """Random (one-ball) states incl. done envs and every dx/dy, one step each."""
    from environment.parallel_breakout import BreakoutEnvironment
    g = np.random.Generator(np.random.PCG64(SEED))
    res = {}
    for tag, (B, H, W) in {"16x20": (4096, 16, 20), "84x84": (512, 84, 84)}.items():
        s = np.zeros((B, 3, H, W), np.float32)
        # bricks: pairs-aligned most of the time, random bits sometimes, rows 0..H-3
        rows = H - 2
        pair = g.random((B, rows, W // 2)) < 0.5
        s[:, 2, :rows, :] = np.repeat(pair, 2, axis=2)
        rnd = g.random(B) < 0.25
        s[rnd, 2, :rows, :] = (g.random((int(rnd.sum()), rows, W)) < 0.5)
        empty = g.random(B) < 0.1
        s[empty, 2] = 0
        # paddle: contiguous 6 at a random column, sometimes absent, sometimes random bits
        pc = g.integers(0, W - 6 + 1, B)
        for b in range(B):
            m = g.random()
            if m < 0.8:
                s[b, 0, H - 1, pc[b]:pc[b] + 6] = 1
            elif m < 0.9:
                s[b, 0, H - 1] = g.random(W) < 0.3
        by = g.integers(0, H, B)
        bx = g.integers(0, W, B)
        # bias some balls to the interesting rows (0, 1, bricks, paddle row, edges)
        sel = g.random(B)
        by = np.where(sel < 0.15, 0, by)
        by = np.where((sel >= 0.15) & (sel < 0.3), H - 1, by)
        by = np.where((sel >= 0.3) & (sel < 0.45), g.integers(0, 4, B), by)
        bx = np.where(g.random(B) < 0.2, g.choice([0, W - 1], B), bx)
        s[np.arange(B), 1, by, bx] = 1
        dx = g.choice([-1, 0, 1], B, p=[0.45, 0.1, 0.45]).astype(np.int64)
        dy = g.choice([-1.0, 0.0, 1.0], B, p=[0.45, 0.1, 0.45]).astype(np.float32)
        # near-win states: a single brick pair exactly where the ball moves next
        win = np.nonzero(g.random(B) < 0.1)[0]
        for b in win:
            nx = bx[b] + dx[b]
            if nx < 0 or nx >= W:
                nx = bx[b] - dx[b]
            ny = int(by[b] + dy[b])
            if 0 <= ny < H - 2:
                s[b, 2] = 0
                s[b, 2, ny, nx - nx % 2: nx - nx % 2 + 2] = 1
        done = g.random(B) < 0.15
        action = g.integers(0, 3, B)
        e = BreakoutEnvironment({**cfg["environment"], "n_parallel": B})
        e.height, e.width = H, W
        e.ball_dx = torch.from_numpy(dx.copy())
        e.ball_dy = torch.from_numpy(dy.copy())
        dm = torch.from_numpy(done.copy())
        ns, r, d2, v = e.step(torch.from_numpy(s.copy()), torch.from_numpy(action), dm)
        assert d2 is dm
        res[tag] = dict(B=B, H=H, W=W, state=pack_state(s), dx=dx, dy=dy, done=done, action=action,
                        next_state=pack_state(ns), reward=r.numpy(), next_done=d2.numpy(), valid=v.numpy(),
                        next_dx=e.ball_dx.numpy(), next_dy=e.ball_dy.numpy())
        np.savez_compressed(os.path.join(HERE, f"envfuzz_{tag}.npz"), **res[tag])
        print("fuzz", tag, "rewards", np.unique(r.numpy(), return_counts=True))


# --------------------------------------------------------------------------------------
def small_model_cfg(cfg):
    m = {**cfg["model"]}
    m["latent_channels"] = [64, 64]
    m["state_history_length"] = 4
    m["representation_network"] = {"num_res_blocks": [1, 1, 1], "activation": "relu"}
    m["dynamics_network"] = {"num_res_blocks": 2, "num_actions": 3, "activation": "relu"}
    m["prediction_network"] = {"num_res_blocks": 2, "num_actions": 3, "activation": "relu"}
    m["device"] = "cpu"
    return m


def load_agent(mcfg, seed):
    reference_modules()
    from src.networks import MuZeroAgent
    agent = MuZeroAgent(mcfg)
    sd = init_state_dict(mcfg, seed)
    agent.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    agent.eval_mode()
    return agent


def make_nets(cfg):
    from utils import ScalarTransforms
    g = np.random.Generator(np.random.PCG64(SEED + 1))
    for tag, mcfg, B in (("full", {**cfg["model"], "device": "cpu"}, 3), ("small", small_model_cfg(cfg), 6)):
        L = mcfg["state_history_length"]
        agent = load_agent(mcfg, SEED)
        st = ScalarTransforms(mcfg)
        # realistic rep input: gray codes {0,.3,.6,1} frames + a/3 action planes
        lut = np.array([0, 0.3, 0.6, 1.0], np.float32)
        frames = lut[g.integers(0, 4, (B, L, 16, 20)) * (g.random((B, L, 16, 20)) < 0.3)]
        acts = g.integers(0, 3, (B, L))
        planes = np.broadcast_to((acts.astype(np.float32) / np.float32(3))[:, :, None, None], (B, L, 16, 20))
        x = np.concatenate([frames, planes], axis=1).astype(np.float32)
        act = g.integers(0, 3, B)
        with torch.no_grad():
            h = agent.create_hidden_state_root(torch.from_numpy(x))
            raw = agent.rep_net(torch.from_numpy(x))
            p0, v0 = agent.evaluate_state(h)
            planes_a = torch.nn.functional.one_hot(torch.from_numpy(act), 3).float().view(B, 3, 1, 1).expand(-1, -1, 4, 5)
            h1, r1 = agent.hidden_state_transition(h, planes_a)
            p1, v1 = agent.evaluate_state(h1)
            dv0 = st.inverted_softmax_expectation(v0)
            dr1 = st.inverted_softmax_expectation(r1)
            dv1 = st.inverted_softmax_expectation(v1)
        np.savez_compressed(os.path.join(HERE, f"nets_{tag}.npz"), weight_seed=SEED, x=x, action=act,
                            rep_raw=raw.numpy(), h=h.numpy(), p0=p0.numpy(), v0=v0.numpy(), h1=h1.numpy(),
                            r1=r1.numpy(), p1=p1.numpy(), v1=v1.numpy(), dv0=dv0.numpy(), dr1=dr1.numpy(),
                            dv1=dv1.numpy(), pi0=torch.softmax(p0, 1).numpy(), pi1=torch.softmax(p1, 1).numpy())
        print("nets", tag, "h range", float(h.min()), float(h.max()), "v0", dv0.numpy()[:3])


# --------------------------------------------------------------------------------------
class SearchInjector:
    """Patches src.mcts: Dirichlet -> noise rows, randint -> keyed tie-break stream,
    and records decoded outputs in call order."""

    def __init__(self, seed):
        reference_modules()
        import src.mcts as mm
        self.mm, self.seed = mm, seed
        self.search_id = -1
        self.cur_env = 0
        self.calls = None
        self.noise = None  # callable(search_id, B) -> (B,3)
        self.dir_calls = 0
        self.rec_softmax, self.rec_ise, self.rec_leaf = [], [], []
        inj = self

        class _Dir:
            def __init__(self, conc):
                pass

            def sample(self):
                b = inj.dir_calls
                inj.dir_calls += 1
                return torch.from_numpy(inj.cur_noise[b].astype(np.float32))

        def randint(high, size, **kw):
            env = inj.cur_env
            k = inj.calls[env]
            inj.calls[env] += 1
            j = R.randbelow(env, R.STREAM_TIE, inj.search_id, k, inj.seed, high)
            return torch.tensor([int(j)])

        def softmax(x, dim):
            out = torch.softmax(x, dim=dim)
            inj.rec_softmax.append(out.detach().numpy().copy())
            return out

        mm.torch = Proxy(torch, randint=randint, softmax=softmax,
                         distributions=Proxy(torch.distributions, Dirichlet=_Dir))
        Base = mm.MCTSSearchVec

        class Search(Base):
            def search(self, hidden_state, action_mask, training_iteration):
                B = hidden_state.shape[0]
                inj.search_id += 1
                inj.calls = [0] * B
                inj.dir_calls = 0
                inj.cur_noise = inj.noise(inj.search_id, B)
                inj.rec_softmax, inj.rec_ise, inj.rec_leaf = [], [], []
                ise = self.scalar_transforms.inverted_softmax_expectation

                def rec_ise(x):
                    out = ise(x)
                    inj.rec_ise.append(out.detach().numpy().copy())
                    return out

                self.scalar_transforms.inverted_softmax_expectation = rec_ise
                try:
                    return super().search(hidden_state, action_mask, training_iteration)
                finally:
                    del self.scalar_transforms.inverted_softmax_expectation

            def ucb_action(self, subtree, action_mask, idx):
                inj.cur_env = idx
                return super().ucb_action(subtree, action_mask, idx)

            def _backup(self, trees, last_nodes, trajectories, *a, **k):
                inj.rec_leaf.append((np.array([ln[1] for ln in last_nodes]),
                                     np.array([len(t) + 1 for t in trajectories])))
                return super()._backup(trees, last_nodes, trajectories, *a, **k)

        self.Search = Search


def dirichlet_noise(search_id, B):
    g = np.random.Generator(np.random.PCG64([SEED, 99, search_id]))
    return g.dirichlet([0.25, 0.25, 0.25], size=B).astype(np.float32)


def make_mcts(cfg):
    from utils import ScalarTransforms
    g = np.random.Generator(np.random.PCG64(SEED + 2))
    mcfg = small_model_cfg(cfg)
    agent = load_agent(mcfg, SEED)
    st = ScalarTransforms(mcfg)
    inj = SearchInjector(SEED)
    inj.noise = dirichlet_noise
    for tag, (B, S) in {"b16_s50": (16, 50), "b4_s200": (4, 200)}.items():
        c = {**cfg, "num_simulations": S}
        search = inj.Search(c, agent, st)
        x = g.random((B, 2 * mcfg["state_history_length"], 16, 20)).astype(np.float32)
        with torch.no_grad():
            h = agent.create_hidden_state_root(torch.from_numpy(x))
            values, counts = search.search(h, torch.ones(B, 3), 0)
        sm, ise = inj.rec_softmax, inj.rec_ise
        assert len(sm) == S + 1 and len(ise) == 1 + 2 * S
        d = dict(B=B, S=S, search_id=inj.search_id, seed=SEED, noise=inj.cur_noise,
                 v_root=ise[0], pi_root=sm[0],
                 r=np.stack(ise[1::2]), v=np.stack(ise[2::2]), pi=np.stack(sm[1:]),
                 counts=counts.numpy(), values=values.numpy(),
                 leaf_action=np.stack([a for a, _ in inj.rec_leaf]), depth=np.stack([d for _, d in inj.rec_leaf]),
                 h=h.numpy())
        np.savez_compressed(os.path.join(HERE, f"mcts_{tag}.npz"), **d)
        print("mcts", tag, "counts[:4]", counts.numpy()[:4].tolist(), "max depth", d["depth"].max(),
              "values[:4]", values.numpy()[:4])


# --------------------------------------------------------------------------------------
def make_acting(cfg, B=4, temperature=1.0, name="acting_small_b4"):
    """One reference `_acting_stage` episode (B=4, small nets) with injected RNG."""
    reference_modules()
    import train_torch as tt
    mcfg = small_model_cfg(cfg)
    c = {**cfg, "n_parallel": B, "model": mcfg, "num_episodes": 1,
         "environment": {**cfg["environment"], "n_parallel": B}}
    inj_reset = ResetInjector(SEED)
    Env = patched_env_class(inj_reset)
    sinj = SearchInjector(SEED)
    sinj.noise = dirichlet_noise
    ncat = [0]

    class InjCategorical:
        def __init__(self, probs):
            self.p = probs.detach().numpy().astype(np.float32)

        def sample(self):
            k = ncat[0]
            ncat[0] += 1
            env, step = k % B, k // B
            u = R.uniform(np.array([env]), R.STREAM_SAMPLE, step, 0, SEED)[0]
            cdf, chosen, last = np.float32(0), -1, 0
            for a in range(3):
                if self.p[a] > 0:
                    last = a
                cdf = np.float32(cdf + self.p[a])
                if chosen < 0 and u < cdf:
                    chosen = a
            return torch.tensor(chosen if chosen >= 0 else last)

    tt.torch = Proxy(torch, distributions=Proxy(torch.distributions, Categorical=InjCategorical))
    tt.get_class = lambda mod, name: {"MCTSSearchVec": sinj.Search, "BreakoutEnvironment": Env}.get(
        name, getattr(__import__(mod, fromlist=[name]), name))
    sys_ = tt.RLSystem(c)
    sd = init_state_dict(mcfg, SEED)
    sd_t = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
    sys_.mu_zero_target.load_state_dict(sd_t)
    sys_.mu_zero.load_state_dict(sd_t)
    sys_.mu_zero_target.eval_mode()
    sys_.temperature = temperature
    state, _ = sys_.environment.reset()
    sys_._pad_initial_state(sys_.convert_to_grayscale(state))
    sys_._run_episode(state)
    trajs = sys_.observation_trajectories
    lens = [t.length for t in trajs]
    L = mcfg["state_history_length"]
    T = max(lens)
    acts = np.full((B, T), -1, np.int64)
    frames = np.zeros((B, T, 16, 20), np.float32)
    rews = np.zeros((B, T), np.float32)
    cnts = np.zeros((B, T, 3), np.int64)
    vals = np.zeros((B, T), np.float32)
    for b, t in enumerate(trajs):
        n = t.length
        acts[b, :n] = [int(a) for a in t.actions[L:]]
        frames[b, :n] = np.stack([s.numpy().reshape(16, 20) for s in t.states[L - 1:]])
        rews[b, :n] = [float(r) for r in t.rewards[L:]]
        cnts[b, :n] = np.stack([v.numpy() for v in t.visit_counts[L:]])
        vals[b, :n] = [float(v) for v in t.values[L:]]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), seed=SEED, B=B, lengths=np.array(lens), temperature=temperature,
                        actions=acts, frames=frames, rewards=rews, counts=cnts, values=vals,
                        n_searches=sinj.search_id + 1,
                        noise=np.stack([dirichlet_noise(i, B) for i in range(sinj.search_id + 1)]))
    print("acting", "lengths", lens, "reward sums", [float(t.reward_sum) for t in trajs])


def reference_modules():
    """The build ships regular packages `src`, `environment`, `utils`, `replay_buffer`
    (muzero-breakout_amd/) that would shadow the reference's modules of the same names: import the
    reference's with the build off the path (idempotent)."""
    if getattr(reference_modules, "_done", False):
        return
    saved = sys.path[:]
    sys.path = [q for q in sys.path if not q.rstrip("/").endswith("muzero-breakout_amd")]
    names = ("src", "utils", "train_torch", "environment", "replay_buffer")
    for m in [m for m in sys.modules if m in names or any(m.startswith(n + ".") for n in names)]:
        del sys.modules[m]
    import train_torch  # noqa: F401
    import src.mcts  # noqa: F401
    import environment.parallel_breakout  # noqa: F401
    sys.path = saved
    reference_modules._done = True


def temperature_schedule(iterations=700):
    """RLSystem.train (train_torch.py:129-132): once training_iteration > 10 every iteration does
    `self.temperature *= 0.996; self.temperature = max(self.temperature, 0.1)` (Python floats).
    Entry k = the temperature after k decays."""
    t, out = 1.0, [1.0]
    for _ in range(iterations):
        t *= 0.996
        t = max(t, 0.1)
        out.append(t)
    return out


def make_sampling(cfg):
    """The reference's temperature step (train_torch.py:192-193 `visit_counts ** (1/self.temperature)`,
    `/ visit_counts_temp.sum(dim=1, keepdim=True)`) evaluated by torch on this CPU on whole int64
    (B, 3) batch tensors, for temperatures of the reference's own schedule, plus the injected inverse-CDF
    choice the acting fixtures use. Batch sizes cover every lane class of torch's CPU pow: B = 4096
    (3B % 32 == 0: all SLEEF vector lanes), 1029 (15 scalar tail lanes), 12 (4 tail), 2 (all tail)."""
    sched = temperature_schedule()
    ks = [0, 1, 2, 3, 10, 37, 100, 150, 250, 400, 500, 573, 574, 575, 700]
    temps = [sched[k] for k in ks] + [0.5, 0.25, 2.0 / 3.0]
    g = np.random.Generator(np.random.PCG64(SEED + 11))
    out = dict(seed=SEED, temps=np.array(temps, np.float64), sched_k=np.array(ks + [-1, -1, -1]),
               vec_block=32, cpu_capability=torch.backends.cpu.get_cpu_capability())
    for name, B, S in (("b4096", 4096, 50), ("b1029", 1029, 200), ("b12", 12, 50), ("b2", 2, 50)):
        p = g.dirichlet([0.3, 0.3, 0.3], B)
        counts = np.stack([g.multinomial(S, p[b]) for b in range(B)]).astype(np.int64)
        counts[: min(B, 8)] = np.array([[S, 0, 0], [0, S, 0], [0, 0, S], [S - 1, 1, 0], [1, 0, S - 1],
                                        [S // 3, S // 3, S - 2 * (S // 3)], [0, S // 2, S - S // 2],
                                        [S - 2, 1, 1]])[: min(B, 8)]
        out[f"{name}/counts"] = counts
        vc = torch.from_numpy(counts)
        for i, T in enumerate(temps):
            vt = vc ** (1 / T)                                   # train_torch.py:192
            probs = vt / vt.sum(dim=1, keepdim=True)              # train_torch.py:193
            u = R.uniform(np.arange(B), R.STREAM_SAMPLE, i, 0, SEED)
            pr = probs.numpy().astype(np.float32)
            act = np.zeros(B, np.int64)
            for b in range(B):  # the acting fixtures' injected Categorical.sample (inverse CDF)
                cdf, chosen, last = np.float32(0), -1, 0
                for a in range(3):
                    if pr[b, a] > 0:
                        last = a
                    cdf = np.float32(cdf + pr[b, a])
                    if chosen < 0 and u[b] < cdf:
                        chosen = a
                act[b] = chosen if chosen >= 0 else last
            out[f"{name}/t{i}/pow"] = vt.numpy()
            out[f"{name}/t{i}/probs"] = pr
            out[f"{name}/t{i}/action"] = act
    # the pow alone over every count 0..1023 and every schedule exponent (4096-element tensors: all
    # vector lanes; and the same values as 31-element tensors: all scalar lanes), as checksums
    base = torch.arange(1024, dtype=torch.int64)
    uniq = sorted(set(sched))
    ex_vec, ex_sc = [], []
    for T in uniq:
        v = (base.repeat(4) ** (1 / T))[:1024].numpy()
        s = torch.cat([(base[i:i + 31] ** (1 / T)) for i in range(0, 1024, 31)]).numpy()
        ex_vec.append(v.view(np.uint32).astype(np.uint64).sum())
        ex_sc.append(s.view(np.uint32).astype(np.uint64).sum())
    out["sched_temps"] = np.array(uniq, np.float64)
    out["sched_pow_vec_u32sum"] = np.array(ex_vec, np.uint64)
    out["sched_pow_scalar_u32sum"] = np.array(ex_sc, np.uint64)
    np.savez_compressed(os.path.join(HERE, "sampling.npz"), **out)
    print("sampling", len(temps), "temperatures;", torch.backends.cpu.get_cpu_capability())


def make_acting_temperature(cfg):
    """One reference `_run_episode` (B = 12, small nets) at a decayed temperature of the reference's
    schedule (150 decays, T ~ 0.548): 3B = 36 elements -> 32 SLEEF vector lanes + 4 scalar lanes."""
    make_acting(cfg, B=12, temperature=temperature_schedule()[150], name="acting_small_b12_t150")


def make_test_sim(cfg):
    """RLSystem.run_test_simulation(batch=2) (train_torch.py:530-610) with injected RNG, small nets,
    a learner net (representation) different from the target net (search), n_parallel = batch = 2
    (the reference resets the whole env batch, :541, and steps it with `batch` actions, :581: only
    n_parallel == batch runs). Records every ObservationTrajectory it builds, the frames it logs
    (env 0, :603-605), and its per-step visit counts and actions."""
    reference_modules()
    import train_torch as tt
    mcfg = small_model_cfg(cfg)
    B = 2
    c = {**cfg, "n_parallel": B, "model": mcfg, "environment": {**cfg["environment"], "n_parallel": B}}
    inj_reset = ResetInjector(SEED + 3)
    Env = patched_env_class(inj_reset)
    sinj = SearchInjector(SEED + 3)
    sinj.noise = dirichlet_noise
    ncat = [0]
    probs_log = []

    class InjCategorical:
        def __init__(self, probs):
            self.p = probs.detach().numpy().astype(np.float32)
            probs_log.append(self.p.copy())

        def sample(self):
            k = ncat[0]
            ncat[0] += 1
            env, step = k % B, k // B
            u = R.uniform(np.array([env]), R.STREAM_SAMPLE, step, 0, SEED + 3)[0]
            cdf, chosen, last = np.float32(0), -1, 0
            for a in range(3):
                if self.p[a] > 0:
                    last = a
                cdf = np.float32(cdf + self.p[a])
                if chosen < 0 and u < cdf:
                    chosen = a
            return torch.tensor(chosen if chosen >= 0 else last)

    trajs = []

    class RecTraj(tt.ObservationTrajectory):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            trajs.append(self)

    images = []

    class Writer:
        def add_image(self, tag, frame, global_step=None, dataformats=None):
            images.append(np.asarray(frame).copy())

        def __getattr__(self, name):
            return lambda *a, **k: None

    tt.torch = Proxy(torch, distributions=Proxy(torch.distributions, Categorical=InjCategorical))
    tt.ObservationTrajectory = RecTraj
    tt.get_class = lambda mod, name: {"MCTSSearchVec": sinj.Search, "BreakoutEnvironment": Env}.get(
        name, getattr(__import__(mod, fromlist=[name]), name))
    sys_ = tt.RLSystem(c)
    sys_.filewriter = Writer()
    sd_t = {k: torch.from_numpy(np.asarray(v)) for k, v in init_state_dict(mcfg, SEED + 4).items()}
    sd_l = {k: torch.from_numpy(np.asarray(v)) for k, v in init_state_dict(mcfg, SEED + 5).items()}
    sys_.mu_zero_target.load_state_dict(sd_t)
    sys_.mu_zero.load_state_dict(sd_l)
    sys_.mu_zero_target.eval_mode()
    sys_.run_test_simulation(B)
    L = mcfg["state_history_length"]
    n = trajs[0].length
    assert all(t.length == n for t in trajs)
    out = dict(seed=SEED + 3, B=B, target_seed=SEED + 4, learner_seed=SEED + 5, n_steps=n,
               actions=np.array([[int(a) for a in t.actions] for t in trajs]),
               rewards=np.array([[float(r) for r in t.rewards[L:]] for t in trajs], np.float32),
               counts=np.stack([np.stack([np.asarray(v) for v in t.visit_counts[L:]]) for t in trajs]).astype(np.int64),
               values=np.array([[float(v) for v in t.values[L:]] for t in trajs], np.float32),
               states=np.stack([np.stack([np.asarray(s).reshape(16, 20) for s in t.states[L - 1:]]) for t in trajs]),
               env0_frames=np.stack(images).reshape(len(images), 16, 20) if images else np.zeros((0, 16, 20), np.float32),
               probs=np.stack(probs_log).reshape(-1, B, 3),
               noise=np.stack([dirichlet_noise(i, B) for i in range(sinj.search_id + 1)]))
    np.savez_compressed(os.path.join(HERE, "test_sim_b2.npz"), **out)
    print("test_sim steps", n, "env0 frames", len(images), "reward sums", [float(t.reward_sum) for t in trajs])


def make_replay(cfg):
    """ReplayBuffer.save_observation_trajectory on seeded synthetic trajectories (reference
    ObservationTrajectory objects padded like _pad_initial_state), small max_length so the
    FIFO eviction runs; every window's getters are stored."""
    import replay_buffer as rb
    K, hist = cfg["num_unroll_steps"], cfg["model"]["state_history_length"]
    H, W = 16, 20
    rng = np.random.default_rng(SEED)
    # the grayscale value set of convert_to_grayscale (train_torch.py:334-358) over the 3 planes
    gray = np.unique(np.array([min(max(np.float32(np.float32(0.3) * p + np.float32(1.0) * b) + np.float32(0.6) * k, 0),
                                   1) for p in (0, 1) for b in (0, 1) for k in (0, 1)], np.float32))
    lengths = [3, 12, 6, 40, 7, 25, 8]  # 3 <= K: no windows; the rest overflow max_length=60
    max_length, nsum = 60, 24
    buf = rb.ReplayBuffer(hist, K, max_length, cfg["discount_factor"], nsum)
    n = len(lengths)
    T = max(lengths)
    acts = np.zeros((n, T), np.int64)
    frames = np.zeros((n, T, H, W), np.float32)
    frame0 = np.zeros((n, H, W), np.float32)
    rews = np.zeros((n, T), np.float32)
    cnts = np.zeros((n, T, 3), np.int64)
    vals = np.zeros((n, T), np.float32)
    for i, L in enumerate(lengths):
        frame0[i] = gray[rng.integers(0, 5, (H, W))]
        t = rb.ObservationTrajectory(actions=[0 for _ in range(hist)],
                                     states=[torch.from_numpy(frame0[i].reshape(1, H, W)) for _ in range(hist - 1)],
                                     rewards=[0 for _ in range(hist)], visit_counts=[torch.zeros(3) for _ in range(hist)],
                                     values=[0.0 for _ in range(hist)], length=0, reward_sum=0)
        for s in range(L):
            a = int(rng.integers(0, 3))
            f = gray[rng.integers(0, 5, (H, W))]
            r = np.float32(rng.choice([-1.0, 0.0, 0.0, 1.0, 5.0, 6.0]))
            c = rng.multinomial(50, [0.3, 0.3, 0.4]).astype(np.int64)
            v = np.float32(rng.normal() * 2)
            acts[i, s], frames[i, s], rews[i, s], cnts[i, s], vals[i, s] = a, f, r, c, v
            t.add_observation(torch.tensor(a), torch.from_numpy(f.reshape(1, H, W)), torch.tensor(r),
                              torch.from_numpy(c), torch.tensor(v))
        buf.save_observation_trajectory(t)
    idx = torch.arange(buf.length)
    out = dict(seed=SEED, K=K, hist=hist, max_length=max_length, num_rewards_to_sum=nsum,
               discount=cfg["discount_factor"], lengths=np.array(lengths), actions=acts, frames=frames,
               frame0=frame0, rewards=rews, counts=cnts, values=vals, n=buf.length,
               past_actions=buf.get_batched_past_actions(idx).numpy(),
               future_actions=buf.get_batched_future_actions(idx).numpy(),
               states=buf.get_batched_states(idx).numpy(),
               b_rewards=buf.get_batched_rewards(idx).numpy(),
               b_counts=buf.get_batched_visit_counts(idx).numpy(),
               b_values=np.stack([v.numpy() for v in buf.value_buffer]),
               targets=buf.get_batched_values(idx).numpy(),
               reward_sums=np.array([float(x) for x in buf.get_reward_sums()], np.float32))
    for k in ("past_actions", "future_actions", "states", "b_rewards", "b_counts", "targets"):
        print("replay", k, out[k].dtype, out[k].shape)
    np.savez_compressed(os.path.join(HERE, "replay.npz"), **out)


def learner_model_cfg(cfg):
    """A narrow learner config: the reference architecture with 32 channels, L = 4."""
    m = small_model_cfg(cfg)
    m["latent_channels"] = [32, 32]
    return m


def learner_minibatch(g, B, L, K):
    """Synthetic replay windows with the replay buffer's value sets (train_torch.py:437-470)."""
    lut = np.array([0, 0.3, 0.6, 1.0], np.float32)
    states = lut[g.integers(0, 4, (B, L, 16, 20)) * (g.random((B, L, 16, 20)) < 0.3)].astype(np.float32)
    past = g.integers(0, 3, (B, L)).astype(np.int64)
    fut = g.integers(0, 3, (B, K)).astype(np.int64)
    rew = g.choice(np.array([-1.0, 0.0, 0.0, 1.0, 5.0, 6.0], np.float32), (B, K)).astype(np.float32)
    val = (g.normal(size=(B, K)) * 2).astype(np.float32)
    cnt = np.stack([g.multinomial(50, [0.3, 0.3, 0.4]) for _ in range(B * K)]).reshape(B, K, 3).astype(np.float32)
    return dict(states=states, past_actions=past, future_actions=fut, rewards=rew, targets=val, counts=cnt)


def reference_train_step(agent, st, mb, mcfg, K):
    """One minibatch of RLSystem._training_stage (train_torch.py:380-407): the reference's own
    _encode_actions, _k_step_rollout, _encode_action_dynamics, loss_fn and Adam step."""
    import train_torch as tt
    L = mcfg["state_history_length"]
    ns = types.SimpleNamespace(mu_zero=agent, K=K, latent_resolution=tuple(mcfg["latent_resolution"]), n_actions=3,
                               state_history_length=L, real_resolution=(16, 20))
    ns._encode_action_dynamics = lambda a, r, n: tt.RLSystem._encode_action_dynamics(ns, a, r, n)
    agent.optimizer.zero_grad()
    states = torch.from_numpy(mb["states"])
    enc = tt.RLSystem._encode_actions(ns, torch.from_numpy(mb["past_actions"]), L, (16, 20))
    pr, pv, pp = tt.RLSystem._k_step_rollout(ns, states, enc, torch.from_numpy(mb["future_actions"]))
    loss, rl, vl, pl = tt.loss_fn(torch.from_numpy(mb["rewards"]), pr, torch.from_numpy(mb["targets"]), pv,
                                  torch.from_numpy(mb["counts"]), pp, st.supports_representation, K)
    loss.backward()
    grads = {k: p.grad.detach().clone().numpy() for k, p in agent.named_parameters()}
    agent.optimizer.step()
    out = dict(loss=np.float32(loss.item()), rl=np.float32(rl.item()), vl=np.float32(vl.item()),
               pl=np.float32(pl.item()), pr=pr.detach().numpy(), pv=pv.detach().numpy(), pp=pp.detach().numpy())
    return out, grads


def make_learner(cfg):
    """Two consecutive reference training minibatches (train mode BN, Adam with weight decay)
    from init_state_dict weights: a narrow config stored in full (logits, losses, every
    gradient, parameters and BN running stats after each step) and the full config at B = 4
    stored as per-tensor checksums plus sampled entries."""
    reference_modules()
    from utils import ScalarTransforms
    from src.networks import MuZeroAgent
    K = cfg["num_unroll_steps"]
    for tag, mcfg, B, full in (("small", learner_model_cfg(cfg), 8, True),
                               ("full", {**cfg["model"], "device": "cpu"}, 4, False)):
        g = np.random.Generator(np.random.PCG64(SEED + 7))
        torch.manual_seed(SEED)
        agent = MuZeroAgent(mcfg)
        sd0 = init_state_dict(mcfg, SEED)
        agent.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd0.items()})
        agent.train_mode()
        st = ScalarTransforms(mcfg)
        L = mcfg["state_history_length"]
        out = dict(seed=SEED, B=B, K=K, lr=mcfg["learning_rate"])
        for step in (1, 2):
            mb = learner_minibatch(g, B, L, K)
            res, grads = reference_train_step(agent, st, mb, mcfg, K)
            after = {k: v.detach().clone().numpy() for k, v in agent.state_dict().items()}
            for k, v in mb.items():
                out[f"s{step}/in/{k}"] = v
            for k in ("loss", "rl", "vl", "pl"):
                out[f"s{step}/{k}"] = res[k]
            if full:
                if step == 1:  # Adam moments after step 1 (reference optimizer state, param order)
                    names = [k for k, _ in agent.named_parameters()]
                    ost = agent.optimizer.state_dict()["state"]
                    for i, k in enumerate(names):
                        out[f"s1/opt/exp_avg/{k}"] = ost[i]["exp_avg"].numpy()
                        out[f"s1/opt/exp_avg_sq/{k}"] = ost[i]["exp_avg_sq"].numpy()
                for k in ("pr", "pv", "pp"):
                    out[f"s{step}/{k}"] = res[k]
                for k, v in grads.items():
                    out[f"s{step}/grad/{k}"] = v
                for k, v in after.items():
                    out[f"s{step}/param/{k}"] = v
            else:
                gs = np.random.Generator(np.random.PCG64(5))
                for k, v in after.items():
                    v0 = np.asarray(sd0[k])
                    flat = v.reshape(-1).astype(np.float64)
                    idx = gs.integers(0, max(flat.size, 1), 16) if flat.size else np.zeros(0, np.int64)
                    out[f"s{step}/idx/{k}"] = idx
                    out[f"s{step}/param_at/{k}"] = v.reshape(-1)[idx]
                    if k in grads:
                        gr = grads[k].reshape(-1).astype(np.float64)
                        out[f"s{step}/grad_at/{k}"] = grads[k].reshape(-1)[idx]
                        out[f"s{step}/grad_sum/{k}"] = np.array([gr.sum(), np.abs(gr).sum(), (gr * gr).sum()])
                        d = flat - v0.reshape(-1).astype(np.float64)
                        out[f"s{step}/delta_sum/{k}"] = np.array([d.sum(), np.abs(d).sum()])
                    else:
                        out[f"s{step}/buf_sum/{k}"] = np.array([flat.sum(), np.abs(flat).sum()])
            if full:  # the reference's own f32 error: its logits / gradients against an f64
                # evaluation of the same algorithm (oracle/learner.py, pinned to the reference in f32)
                from oracle.learner import LearnerOracle
                start = sd0 if step == 1 else {k[len("s1/param/"):]: out[k] for k in out if k.startswith("s1/param/")}
                o64 = LearnerOracle(mcfg, start, K=K, dtype=torch.float64)
                _, lg64, g64 = o64.gradients(mb)
                for k, a in zip(("pr", "pv", "pp"), lg64):
                    out[f"s{step}/err_ref/{k}"] = np.float64(np.abs(res[k].astype(np.float64) - a.numpy()).max())
                for k, gr in grads.items():
                    out[f"s{step}/err_ref/grad/{k}"] = np.float64(np.abs(gr.astype(np.float64) - g64[k].numpy()).max())
            print("learner", tag, "step", step, "loss", float(res["loss"]), float(res["rl"]), float(res["vl"]),
                  float(res["pl"]))
        np.savez_compressed(os.path.join(HERE, f"learner_{tag}.npz"), **out)


# --------------------------------------------------------------------------------------
def make_agent_init(cfg):
    """The reference agent's own random initialisation (networks.py:245-266, MuZeroAgent(cfg) as
    RLSystem.__init__ builds it twice, train_torch.py:86-88) under torch.manual_seed(s): the small
    and the full-width model's state_dicts as per-tensor checksums (f64 sum, sum of |x|, first 4 and
    last elements), for the learner agent and the target agent built right after it."""
    reference_modules()
    from src.networks import MuZeroAgent
    out = {}
    for tag, mcfg in (("small", small_model_cfg(cfg)), ("full", {**cfg["model"], "device": "cpu"})):
        for seed in (42, 7):
            torch.manual_seed(seed)
            agents = [MuZeroAgent(mcfg), MuZeroAgent(mcfg)]  # self.mu_zero, self.mu_zero_target
            for ai, ag in enumerate(agents):
                for k, v in ag.state_dict().items():
                    a = v.detach().cpu().numpy()
                    key = f"{tag}/s{seed}/a{ai}/{k}"
                    f = a.astype(np.float64).reshape(-1)
                    out[key] = np.concatenate([[f.sum(), np.abs(f).sum()], f[:4], f[-1:]])
            print("agent_init", tag, seed, len(agents[0].state_dict()), "tensors")
    np.savez_compressed(os.path.join(HERE, "agent_init.npz"), **out)


if __name__ == "__main__":
    cfg = ref_harness.load_config()
    which = sys.argv[1:] or ["env", "fuzz", "nets", "mcts", "acting", "replay", "learner", "sampling", "acting_t",
                             "test_sim", "agent_init"]
    if "env" in which:
        make_env(cfg)
    if "fuzz" in which:
        make_env_fuzz(cfg)
    if "nets" in which:
        make_nets(cfg)
    if "mcts" in which:
        make_mcts(cfg)
    if "acting" in which:
        make_acting(cfg)
    if "replay" in which:
        make_replay(cfg)
    if "learner" in which:
        make_learner(cfg)
    if "sampling" in which:
        make_sampling(cfg)
    if "acting_t" in which:
        make_acting_temperature(cfg)
    if "test_sim" in which:
        make_test_sim(cfg)
    if "agent_init" in which:
        make_agent_init(cfg)
