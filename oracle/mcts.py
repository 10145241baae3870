"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of `src/mcts.py::MCTSSearchVec` (per-env dict trees, Python loops, as
the reference) with every f32 operation in the reference's order, and with the two
random sources injected:
  * Dirichlet root noise (mcts.py:114) -> `noise[B,3]` argument,
  * ucb tie-break `best[torch.randint(len(best))]` (mcts.py:297) ->
    best[randbelow(len(best))] from the keyed Philox stream
    (env, STREAM_TIE, search_id, k), k = per-env ucb_action call counter.
Scalars follow torch's semantics for f32 0-d tensors with Python scalars:
f32 op f32(scalar) (verified against the reference).

`model` supplies network outputs already decoded exactly as the reference does on
its device: `root(h) -> (v[B] f32, pi[B,3] f32)` and
`expand(parent_latents, actions) -> (latents, r[B], v[B], pi[B,3])`.
"""
import math

import numpy as np

from . import rng as R

f32 = np.float32


class MCTSOracle:
    def __init__(self, cfg, model, seed=0):
        self.num_simulations = cfg["num_simulations"]  # mcts.py:13
        self.actions = list(cfg["actions"])
        self.c1 = cfg["search"]["c1"]
        self.c2 = cfg["search"]["c2"]
        self.discount = cfg["search"]["discount_factor"]
        self.noise_weight = 0.175  # mcts.py:22 (train loop sets 0.1 at iteration 100)
        self.model = model
        self.seed = seed
        self.trace = None  # optional list of per-sim (parent name, action) for debugging

    # mcts.py:281-298
    def ucb_action(self, subtree, env, ctx):
        n = sum(int(subtree[a]["N"]) for a in self.actions)
        log_term = (n + self.c2 + 1) / self.c2
        sq = f32(math.sqrt(n))
        cterm = f32(self.c1 + math.log(log_term))
        ucb = []
        for a in self.actions:
            e = subtree[a]
            t = f32(e["P"] * sq)
            t = f32(t / f32(1 + e["N"]))
            t = f32(t * cterm)
            ucb.append(f32(f32(e["Q"]) + t))
        ucb = np.array(ucb, dtype=np.float32)
        mx = ucb.max()
        best = np.nonzero(ucb == mx)[0]
        k = ctx["calls"][env]
        ctx["calls"][env] += 1
        j = int(R.randbelow(env + ctx["env_offset"], R.STREAM_TIE, ctx["search_id"], k, self.seed, len(best)))
        return int(best[j])

    def search(self, hidden_state, noise, search_id, env_offset=0):
        """mcts.py:24-71. hidden_state (B, ...) ndarray, noise (B,3) f32."""
        B = hidden_state.shape[0]
        S = self.num_simulations
        ctx = {"calls": [0] * B, "search_id": search_id, "env_offset": env_offset}
        trees = [{"state_0": {0: {"N": 0, "Q": f32(0)}, 1: {"N": 0, "Q": f32(0)}, 2: {"N": 0, "Q": f32(0)},
                              3: {"N": 0, "Q": f32(0)}, "state": hidden_state[b], "value": None,
                              "expanded": False}} for b in range(B)]
        # _expand_root_nodes mcts.py:91-134
        v_root, pi_root = self.model.root(hidden_state)
        w_pol = f32(1 - self.noise_weight)
        w_noise = f32(self.noise_weight)
        expand_buffer, last_nodes, trajectories = [], [], []
        for b in range(B):
            t = trees[b]
            t["state_0"]["value"] = f32(v_root[b])
            t["state_0"]["expanded"] = True
            for a in self.actions:
                child = f"state_0_{a}"
                t["state_0"][a]["P"] = f32(f32(w_pol * f32(pi_root[b, a])) + f32(w_noise * f32(noise[b, a])))
                t["state_0"][a]["next_state"] = child
                t[child] = {"expanded": False}
            a = self.ucb_action(t["state_0"], b, ctx)
            expand_buffer.append(hidden_state[b])
            last_nodes.append(("state_0", a, t["state_0"][a]["next_state"]))
            trajectories.append([])
        for sim in range(S):
            if sim > 0:
                trajectories, expand_buffer, last_nodes = self._select(trees, B, ctx)
            if self.trace is not None:
                self.trace.append([(ln[0], ln[1]) for ln in last_nodes])
            acts = np.array([ln[1] for ln in last_nodes], dtype=np.int64)
            lat, r, v, pi = self.model.expand(np.stack(expand_buffer), acts)
            self._backup(trees, last_nodes, trajectories, lat, r, v, pi, sim, B)
        values = np.array([float(trees[b]["state_0"]["value"]) / S for b in range(B)], dtype=np.float64).astype(np.float32)
        counts = np.array([[trees[b]["state_0"][a]["N"] for a in self.actions] for b in range(B)], dtype=np.int64)
        return values, counts

    # mcts.py:136-182
    def _select(self, trees, B, ctx):
        trajectories, expand_buffer, last_nodes = [], [], []
        for b in range(B):
            traj = []
            cur = "state_0"
            sub = trees[b][cur]
            while True:
                a = self.ucb_action(sub, b, ctx)
                prev = cur
                cur = sub[a]["next_state"]
                sub = trees[b][cur]
                if sub["expanded"]:
                    traj.append((prev, a, trees[b][prev][a]["R"]))
                else:
                    trees[b][cur] = {0: {"N": 0}, 1: {"N": 0}, 2: {"N": 0}, 3: {"N": 0},
                                     "state": None, "value": None, "expanded": True}
                    expand_buffer.append(trees[b][prev]["state"])
                    last_nodes.append((prev, a, cur))
                    break
            trajectories.append(traj)
        return trajectories, expand_buffer, last_nodes

    # mcts.py:203-234
    def _backup(self, trees, last_nodes, trajectories, lat, r, v, pi, sim, B):
        disc = f32(self.discount)
        for b in range(B):
            prev, action, cur = last_nodes[b]
            value = f32(v[b])
            trees[b][cur]["state"] = lat[b]
            trees[b][prev][action]["R"] = f32(r[b])
            trees[b][cur]["value"] = value
            for a in self.actions:
                nxt = f"state_{sim + 1}_{a}"
                trees[b][cur][a] = {"N": 0, "Q": f32(0), "P": f32(pi[b, a]), "R": f32(0), "next_state": nxt}
                trees[b][nxt] = {"expanded": False}
            trajectories[b].append((prev, action, f32(r[b])))
            for node, a, rr in reversed(trajectories[b]):
                value = f32(f32(value * disc) + rr)
                trees[b][node]["value"] = f32(trees[b][node]["value"] + value)
                e = trees[b][node][a]
                e["Q"] = f32(f32(f32(e["N"]) * e["Q"]) + value) / f32(e["N"] + 1)
                e["Q"] = f32(e["Q"])
                e["N"] += 1


class ReplayModel:
    """Feeds recorded decoded network outputs (fixture replay mode)."""

    def __init__(self, v_root, pi_root, r, v, pi):
        self.v_root, self.pi_root = v_root, pi_root
        self.r, self.v, self.pi = r, v, pi
        self.sim = 0

    def root(self, h):
        self.sim = 0
        return self.v_root, self.pi_root

    def expand(self, parents, actions):
        s = self.sim
        self.sim += 1
        return parents, self.r[s], self.v[s], self.pi[s]


class NetModel:
    """Runs the oracle nets (f32) and decodes like mcts.py:95-100, 194-199."""

    def __init__(self, sd, mcfg):
        from . import nets
        self.nets = nets
        self.sd, self.mcfg = sd, mcfg

    def root(self, h):
        p, v = self.nets.prediction(h, self.sd, self.mcfg)
        return (self.nets.inverted_softmax_expectation(v, self.mcfg["supports_min"], self.mcfg["supports_max"]),
                self.nets.softmax(p, axis=1))

    def expand(self, parents, actions):
        planes = self.nets.encode_action_planes(actions, self.mcfg["latent_resolution"], 3, parents.dtype)
        h, r = self.nets.dynamics(parents, planes, self.sd, self.mcfg)
        p, v = self.nets.prediction(h, self.sd, self.mcfg)
        smin, smax = self.mcfg["supports_min"], self.mcfg["supports_max"]
        return (h, self.nets.inverted_softmax_expectation(r, smin, smax),
                self.nets.inverted_softmax_expectation(v, smin, smax), self.nets.softmax(p, axis=1))
