"""Latent MCTS on the MI355X path (mirror of src/mcts.py:MCTSSearchVec).

The whole search runs on the device with no host synchronisation, every launch a torch custom op
(`torch.ops.mz`): per simulation the fused dynamics step (`dynamics_`, parent latents gathered from
the node pool by the selected slots) and the fused prediction step that also backs up the
simulation and selects the next leaf (`prediction_tree_`); unfused, one select kernel, the
prediction net and one backup kernel.
The launch sequence is identical for every call of a given (B, S), so the acting loop
can capture it in a HIP graph.
"""
import math
import os

import numpy as np
import torch

from . import _lib as L
from .agent import MuZeroAgent  # noqa: F401  (re-export for the drop-in module)


def ucb_tables(S, c1, c2, device):
    """f32(sqrt(n)) and f32(c1 + log((n + c2 + 1) / c2)) for n = 0..S, evaluated in
    double exactly as mcts.py:285-289 does (math.sqrt / math.log on Python floats)."""
    sq = np.array([math.sqrt(n) for n in range(S + 1)], dtype=np.float64).astype(np.float32)
    ct = np.array([c1 + math.log((n + c2 + 1) / c2) for n in range(S + 1)], dtype=np.float64).astype(np.float32)
    return torch.from_numpy(sq).to(device), torch.from_numpy(ct).to(device)


class TreeState:
    """Device buffers of B search trees with S simulations."""

    def __init__(self, B, S, c1, c2, device):
        self.B, self.S = B, S
        nb = L.lib().mzba_mcts_node_bytes()
        self.nodes = torch.empty(B * (S + 1) * nb, dtype=torch.uint8, device=device)
        self.root_sum = torch.empty(B, dtype=torch.float32, device=device)
        self.calls = torch.empty(B, dtype=torch.int32, device=device)
        self.leaf_parent = torch.empty(B, dtype=torch.int32, device=device)
        self.leaf_action = torch.empty(B, dtype=torch.int32, device=device)
        self.depth = torch.empty(B, dtype=torch.int32, device=device)
        self.path = torch.empty(B * (S + 1), dtype=torch.int32, device=device)
        self.sqrt_tab, self.c_tab = ucb_tables(S, c1, c2, device)
        self.counts = torch.empty(B, 3, dtype=torch.int64, device=device)
        self.values = torch.empty(B, dtype=torch.float32, device=device)
        self.noise = torch.empty(B, 3, dtype=torch.float32, device=device)

    def args(self, env_offset, search_id, seed, ctx=None):
        """Tree arguments of the torch.ops.mz tree ops (csrc/torch_ops.cpp). ctx: optional device
        int32[3] step context (its [0] overrides search_id; graph replay)."""
        return (self.nodes, self.root_sum, self.calls, self.leaf_parent, self.leaf_action, self.depth, self.path,
                self.sqrt_tab, self.c_tab, self.S, env_offset, search_id, seed, ctx)

    # individual kernels, dispatched as torch custom ops -----------------------------------------
    def root(self, tree_args, v_root, pi_root, noise_in, w_pol, w_noise, alpha, w_dev=None):
        L.ops().mcts_root_(*tree_args, v_root, pi_root, noise_in, self.noise, w_pol, w_noise, w_dev, alpha)

    def select(self, tree_args, sim):
        L.ops().mcts_select_(*tree_args, sim)

    def backup(self, tree_args, sim, r, v, pi, gamma):
        L.ops().mcts_backup_(*tree_args, sim, r, v, pi, gamma)

    def results(self, tree_args):
        L.ops().mcts_results_(*tree_args, self.values, self.counts)


class MCTSSearchVec:
    """Drop-in for src/mcts.py:MCTSSearchVec (constructor and `search` signature).

    search(hidden_state (B,C,h,w), action_mask (B,3), training_iteration)
      -> (values f32[B] CPU, visit_counts i64[B,3] CPU), like mcts.py:71.
    `action_mask` and `training_iteration` are accepted and ignored, as in the
    reference (mcts.py:124,157 use ones_like(action_mask)).
    Randomness: Dirichlet root noise and ucb tie-breaks come from the keyed Philox
    stream (seed, global env, search id) — see DESIGN.md §RNG.
    """

    def __init__(self, cfg, mu_zero, scalar_transforms=None, seed=0, env_offset=0):
        self.num_simulations = cfg["num_simulations"]  # mcts.py:13-22
        self.actions = cfg["actions"]
        self.c1 = cfg["search"]["c1"]
        self.c2 = cfg["search"]["c2"]
        self.discount = cfg["search"]["discount_factor"]
        self.mu_zero = mu_zero
        self.scalar_transforms = scalar_transforms
        self.latent_resolution = cfg["latent_resolution"]
        self.dirchlet_alpha = 0.25
        self.noise_weight = 0.175
        self.seed = seed
        self.env_offset = env_offset
        self.search_id = 0
        self._ws = {}

    # workspace per (B, agent) -------------------------------------------------------------
    def workspace(self, B):
        key = (B, id(self.mu_zero), self.mu_zero.dtype)
        ws = self._ws.get(key)
        if ws is None:
            ws = SearchWorkspace(self, B)
            self._ws = {key: ws}
        return ws

    def search(self, hidden_state, action_mask=None, training_iteration=0, noise=None):
        B = hidden_state.shape[0]
        ws = self.workspace(B)
        ws.load_root(hidden_state)
        if noise is not None:  # injected Dirichlet rows (B, 3), any array-like
            noise = torch.as_tensor(np.asarray(noise, dtype=np.float32), device=ws.agent.device).contiguous()
        values, counts = ws.run(self.search_id, noise)
        self.search_id += 1
        return values.cpu(), counts.cpu()


class SearchWorkspace:
    """Buffers + launch sequence of one search over B envs (NHWC latents)."""

    def __init__(self, search, B):
        agent = search.mu_zero
        self.s = search
        self.agent = agent
        dev = agent.device
        p = agent.packed
        self.B, self.S = B, search.num_simulations
        self.n = p.lh * p.lw * p.c1
        self.tree = TreeState(B, self.S, search.c1, search.c2, dev)
        self.pool = torch.empty(B * (self.S + 1) * self.n, dtype=p.tdt, device=dev)
        self.cur = torch.empty(B * self.n, dtype=p.tdt, device=dev)
        self.r = torch.empty(B, dtype=torch.float32, device=dev)
        self.v = torch.empty(B, dtype=torch.float32, device=dev)
        self.pi = torch.empty(B, 3, dtype=torch.float32, device=dev)
        self.runner = agent.runner(B, p.lh * 4, p.lw * 4)
        # backup + next select ride on the fused prediction launch (MZBA_TREE_FUSION=0: separate kernels)
        self.use_tree_fusion = os.environ.get("MZBA_TREE_FUSION", "1") != "0"
        # fused steps: latents straight from / to their node-pool slots (MZBA_POOL_SLOTS=0: through `cur`,
        # the round-3 second-session form, for A/B runs)
        self.use_pool_slots = os.environ.get("MZBA_POOL_SLOTS", "1") != "0"

    def load_root(self, hidden_state):
        """NCHW (B,C,h,w) latent -> pool slot 0 (NHWC)."""
        p = self.agent.packed
        B = self.B
        x = hidden_state.to(self.agent.device).permute(0, 2, 3, 1).reshape(B, self.n).to(p.tdt)
        self.pool.view(B, self.S + 1, self.n)[:, 0].copy_(x)

    def root_slot(self):
        return self.pool.view(self.B, self.S + 1, self.n)[:, 0]

    def run(self, search_id, noise=None, ctx=None, w_dev=None):
        """mcts.py:24-71 on the device. Root latent must be in pool slot 0. With `ctx` the
        search id is read on the device (HIP-graph replayable launch sequence); `w_dev` (device
        f32[2]) supplies the root mixing weights (f32(1 - noise_weight), f32(noise_weight))."""
        s = self.s
        B, S, n = self.B, self.S, self.n
        ta = self.tree.args(s.env_offset, search_id, s.seed, ctx)
        rn = self.runner
        slots = self.pool.view(B, S + 1, n)  # node pool: slot 0 the root, slot s + 1 the node of simulation s
        fused = rn.fused_ok() and self.use_tree_fusion
        direct = fused and self.use_pool_slots
        # the fused steps read each latent from its node-pool slot and the dynamics step writes the new
        # latent there only (no copy into `cur`: one latent write per env and simulation, not two)
        rn.prediction(slots[:, 0] if direct else self._root_copy(slots), self.pi, self.v)  # _expand_root_nodes mcts.py:95-100
        w_pol = float(np.float32(1 - s.noise_weight))
        w_noise = float(np.float32(s.noise_weight))
        self.tree.root(ta, self.v, self.pi, noise, w_pol, w_noise, s.dirchlet_alpha, w_dev)
        gamma = float(np.float32(s.discount))
        env_stride = (S + 1) * n
        for sim in range(S):
            if sim > 0 and not fused:
                self.tree.select(ta, sim)
            rn.dynamics(self.pool, self.tree.leaf_action, None if direct else self.cur, self.r,
                        slot=self.tree.leaf_parent, env_stride=env_stride, slot_stride=n, pool=self.pool,
                        pool_env_stride=env_stride, pool_slot=sim + 1)
            if fused:  # prediction + backup(sim) + select(sim + 1) in one launch
                rn.prediction(slots[:, sim + 1] if direct else self.cur, self.pi, self.v, tree=(ta, sim, gamma, self.r))
            else:
                rn.prediction(self.cur, self.pi, self.v)
                self.tree.backup(ta, sim, self.r, self.v, self.pi, gamma)
        self.tree.results(ta)
        return self.tree.values, self.tree.counts

    def _root_copy(self, slots):
        """The root latents contiguous in `cur` (the unfused launches read contiguous latents)."""
        self.cur.view(self.B, self.n).copy_(slots[:, 0])
        return self.cur


def replay_search(B, S, cfg, v_root, pi_root, noise, r, v, pi, seed, search_id, env_offset=0, device="cuda"):
    """Tree kernels driven by recorded decoded network outputs (fixture replay mode):
    the same select/backup/results launches as SearchWorkspace.run, without nets."""
    L.require_gpu()
    t = TreeState(B, S, cfg["search"]["c1"], cfg["search"]["c2"], device)
    dv = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=device)  # noqa: E731
    ta = t.args(env_offset, search_id, seed)
    t.root(ta, dv(v_root), dv(pi_root), dv(noise), float(np.float32(1 - 0.175)), float(np.float32(0.175)), 0.25)
    gamma = float(np.float32(cfg["search"]["discount_factor"]))
    leaf = np.zeros((S, B), dtype=np.int64)
    for sim in range(S):
        if sim > 0:
            t.select(ta, sim)
        leaf[sim] = t.leaf_action.cpu().numpy()
        t.backup(ta, sim, dv(r[sim]), dv(v[sim]), dv(pi[sim]), gamma)
    t.results(ta)
    return t.values.cpu().numpy(), t.counts.cpu().numpy(), leaf
