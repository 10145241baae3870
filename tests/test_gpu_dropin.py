"""The reference's own caller against this build: RLSystem.__init__'s construction sequence
(train_torch.py:86-101) and one whole `_acting_stage` episode (:160-233) driven exactly as the
reference drives it, on the classes `get_class` resolves from this build's drop-in modules.

The reference is not on the GPU box, so the caller's statements are restated here (each block cites
the lines it restates); everything they call is this build's: `src.networks.MuZeroAgent`,
`src.mcts.MCTSSearchVec`, `environment.parallel_breakout.BreakoutEnvironment`, `utils`,
`replay_buffer.ReplayBuffer` / `ObservationTrajectory`.
"""
import numpy as np
import pytest
import torch

from mzba.config import default_config

pytestmark = pytest.mark.gpu


class _RLSystemCalls:
    """The statements of train_torch.py:RLSystem that touch the plugins, in the reference's order."""

    def __init__(self, cfg):
        from utils import get_class, ScalarTransforms
        from replay_buffer import ReplayBuffer
        self.real_resolution = cfg["real_resolution"]
        self.state_history_length = cfg["model"]["state_history_length"]
        self.n_actions = len(cfg["actions"])
        self.K = cfg["num_unroll_steps"]
        self.n_parallel = cfg["n_parallel"]
        self.temperature = 1.0
        self.training_iteration = 0
        # :86-94
        mu_zero_class = get_class("src.networks", cfg["model"]["agent_name"])
        self.mu_zero = mu_zero_class(cfg["model"])
        self.mu_zero_target = mu_zero_class(cfg["model"])
        self.mu_zero_target.load_state_dict(self.mu_zero.state_dict())
        latent_mcts_class = get_class("src.mcts", cfg["search"]["mcts_name"])
        self.scalar_transforms = ScalarTransforms(cfg["model"])
        self.latent_mcts = latent_mcts_class(cfg, self.mu_zero_target, self.scalar_transforms)
        environment_class = get_class(cfg["environment"]["environment_path"], cfg["environment"]["environment_name"])
        self.environment = environment_class(cfg["environment"])
        # :97-98
        for param in self.mu_zero_target.parameters():
            param.requires_grad = False
        # :101
        self.replay_buffer = ReplayBuffer(self.state_history_length, self.K, cfg["replay_buffer_max"],
                                          cfg["discount_factor"], self.n_parallel)
        self.observation_trajectories = []

    # :313-332
    def pad_initial_state(self, initial_state):
        from replay_buffer import ObservationTrajectory
        L = self.state_history_length
        self.observation_trajectories = [
            ObservationTrajectory(actions=[0] * L, states=[initial_state[i] for _ in range(L - 1)], rewards=[0] * L,
                                  visit_counts=[torch.zeros(self.n_actions) for _ in range(L)], values=[0.0] * L,
                                  length=0, reward_sum=0)
            for i in range(self.n_parallel)]

    # :334-358
    @staticmethod
    def convert_to_grayscale(state):
        g = state[:, 0] * 0.3 + state[:, 1] * 1.0 + state[:, 2] * 0.6
        return g.clamp(0, 1).unsqueeze(1)

    # :259-293
    def prepare_mcts_input(self, state, traj):
        L, (h, w) = self.state_history_length, self.real_resolution
        actions = traj.get_actions()[-L:].unsqueeze(0)
        planes = (actions / self.n_actions)[:, :, None, None].expand(-1, -1, h, w)
        planes = (torch.ones((1, L, h, w), device=planes.device) * planes).squeeze(0)
        seq = torch.cat((traj.get_states()[-(L - 1):].view(-1, h, w), state), dim=0)
        return torch.cat((seq, planes), dim=0)

    # :236-257
    def sample_action(self, state, mask):
        x = torch.stack([self.prepare_mcts_input(state[i], t) for i, t in enumerate(self.observation_trajectories)])
        hidden_state = self.mu_zero_target.create_hidden_state_root(x)
        return self.latent_mcts.search(hidden_state, mask, self.training_iteration)

    # :160-233, one episode
    def acting_stage_episode(self, on_step=None):
        self.mu_zero_target.eval_mode()
        initial_state, done = self.environment.reset()
        self.pad_initial_state(self.convert_to_grayscale(initial_state))
        state = initial_state
        done_mask = torch.zeros((state.shape[0]), dtype=torch.bool)
        prev_done_mask = done_mask
        valid_actions = torch.ones((state.shape[0], self.n_actions))
        warp_state = self.convert_to_grayscale(state)
        steps = 0
        while not torch.all(done_mask == True):  # noqa: E712 (the reference's own test)
            if steps > 260:
                break
            value, visit_counts = self.sample_action(warp_state, valid_actions)
            vt = visit_counts ** (1 / self.temperature)
            probs = vt / vt.sum(dim=1, keepdim=True)
            action = torch.zeros(probs.shape[0], dtype=torch.long)
            for i in range(probs.shape[0]):
                action[i] = torch.distributions.Categorical(probs[i]).sample()
            state, reward, done_mask, valid_actions = self.environment.step(state, action, done_mask)
            warp_state = self.convert_to_grayscale(state)
            for i in range(len(self.observation_trajectories)):
                if not prev_done_mask[i]:
                    self.observation_trajectories[i].add_observation(action[i], warp_state[i], reward[i],
                                                                     visit_counts[i], value[i])
            prev_done_mask = done_mask.clone()
            if on_step is not None:
                on_step(steps, value, visit_counts, action, reward, done_mask)
            steps += 1
        for t in self.observation_trajectories:  # :223-225
            if t.length > (self.K + 1):
                self.replay_buffer.save_observation_trajectory(t)
        return steps, self.replay_buffer.get_reward_sums()  # :230


def test_rlsystem_constructs_and_acts_on_this_build():
    """train_torch.py:86-101 then one `_acting_stage` episode (:164-233) with the reference's config.yaml
    values (24 envs, full-width nets, 50 simulations), on the drop-in classes."""
    torch.manual_seed(42)  # train_torch.py set_seed(42)
    cfg = default_config()
    rl = _RLSystemCalls(cfg)
    # the agents start from the reference's random init and the target copies the learner (:87-89)
    sd_l, sd_t = rl.mu_zero.state_dict(), rl.mu_zero_target.state_dict()
    assert list(sd_l) == list(sd_t) and len(sd_l) == 542
    for k in sd_l:
        assert torch.equal(sd_l[k], sd_t[k]), k
    assert all(not p.requires_grad for p in rl.mu_zero_target.parameters())
    assert any(p.requires_grad for p in rl.mu_zero.parameters())
    assert len(list(rl.mu_zero.parameters())) == sum(1 for k in sd_l if not k.endswith(
        ("running_mean", "running_var", "num_batches_tracked")))
    assert rl.mu_zero._packed is None  # the learner agent is never packed: nothing ran on it
    S, B, K = cfg["num_simulations"], cfg["n_parallel"], cfg["num_unroll_steps"]
    seen = []

    def on_step(t, value, counts, action, reward, done):
        assert value.dtype == torch.float32 and value.shape == (B,) and value.device.type == "cpu"
        assert counts.dtype == torch.int64 and counts.shape == (B, 3) and counts.device.type == "cpu"
        assert (counts.sum(1) == S).all(), counts
        assert torch.isfinite(value).all()
        assert reward.device.type == "cpu" and done.device.type == "cpu"
        seen.append((counts.clone(), action.clone(), done.clone()))

    steps, reward_sums = rl.acting_stage_episode(on_step)
    assert 1 <= steps <= 261 and len(seen) == steps
    L = rl.state_history_length
    windows = 0
    for i, t in enumerate(rl.observation_trajectories):
        live = [s for s in range(steps) if s == 0 or not bool(seen[s - 1][2][i])]
        assert t.length == len(live)
        assert len(t.actions) == L + t.length and len(t.states) == L - 1 + t.length
        assert all(s.shape == (1, 16, 20) for s in t.states)
        np.testing.assert_array_equal(np.array([int(a) for a in t.actions[L:]]),
                                      np.array([int(seen[s][1][i]) for s in live]))
        np.testing.assert_array_equal(torch.stack(t.visit_counts[L:]).numpy(),
                                      np.stack([seen[s][0][i].numpy() for s in live]))
        if t.length > K + 1:
            windows += t.length - K + 1
    assert rl.replay_buffer.length == windows
    assert len(reward_sums) == min(B, windows)
