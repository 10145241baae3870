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


def _loss_fn(observed_reward, predicted_reward, bootstrapped_reward, predicted_value, visit_counts, predicted_policy,
             target_transformation, K):
    """train_torch.py:33-66 (loss_fn), restated."""
    import torch.nn.functional as F
    reward_loss = F.kl_div(F.log_softmax(predicted_reward.view(-1, predicted_reward.shape[-1]), dim=-1),
                           target_transformation(observed_reward).view(-1, predicted_reward.shape[-1]),
                           reduction="batchmean")
    value_loss = F.kl_div(F.log_softmax(predicted_value.view(-1, predicted_value.shape[-1]), dim=-1),
                          target_transformation(bootstrapped_reward).view(-1, predicted_value.shape[-1]),
                          reduction="batchmean")
    vcn = visit_counts / visit_counts.sum(dim=-1, keepdim=True)
    policy_loss = F.kl_div(F.log_softmax(predicted_policy.view(-1, predicted_policy.shape[-1]), dim=-1),
                           vcn.view(-1, vcn.shape[-1]), reduction="batchmean")
    return (1 / K) * (reward_loss + value_loss + policy_loss), reward_loss, value_loss, policy_loss


def _training_iteration(mu_zero, scalar_transforms, mb, K, L, latent_resolution, n_actions=3):
    """One iteration of RLSystem._training_stage's loop body (train_torch.py:385-411) on a minibatch already
    drawn from the replay buffer (_prepare_minibatch :454-485): _encode_actions (:279-293), _k_step_rollout
    (:487-528, with _encode_action_dynamics :295-311), loss_fn, loss.backward(), optimizer.step()."""
    import torch.nn.functional as F
    dev = "cuda"
    mu_zero.optimizer.zero_grad()
    with torch.no_grad():
        states = torch.as_tensor(mb["states"], dtype=torch.float32, device=dev)
        B = states.shape[0]
        acts = torch.as_tensor(mb["past_actions"], device=dev)
        ex = (acts / n_actions)[:, :, None, None].expand(-1, -1, 16, 20)
        input_actions_encoded = torch.ones((B, L, 16, 20), device=dev) * ex
    repnet_input = torch.cat((states.view(B, L, 16, 20), input_actions_encoded), dim=1)
    hidden_state = mu_zero.create_hidden_state_root(repnet_input)
    k_step_actions = torch.as_tensor(mb["future_actions"], device=dev)
    pols, vals, rews = [], [], []
    for k in range(K):
        p, v = mu_zero.evaluate_state(hidden_state)
        pols.append(p)
        vals.append(v)
        one_hot = F.one_hot(k_step_actions[:, k], num_classes=n_actions).float()
        a_enc = one_hot.view(B, n_actions, 1, 1).expand(-1, -1, latent_resolution[0], latent_resolution[1])
        hidden_state, r = mu_zero.hidden_state_transition(hidden_state, a_enc)
        rews.append(r)
    pr, pv, pp = torch.stack(rews, 1), torch.stack(vals, 1), torch.stack(pols, 1)
    tt = lambda x: scalar_transforms.supports_representation(torch.as_tensor(x, dtype=torch.float32)).to(dev)  # noqa: E731
    loss, rl, vl, pl = _loss_fn(torch.as_tensor(mb["rewards"]), pr, torch.as_tensor(mb["targets"]), pv,
                                torch.as_tensor(mb["counts"], dtype=torch.float32, device=dev), pp, tt, K)
    loss.backward()
    mu_zero.optimizer.step()
    return (np.array([float(x.detach()) for x in (loss, rl, vl, pl)]), (pr.detach(), pv.detach(), pp.detach()))


def test_training_stage_runs_on_the_dropin_agent():
    """RLSystem._training_stage on this build's MuZeroAgent (train_torch.py:373-411): train_mode(), then the
    reference's own minibatch loop body — zero_grad, _k_step_rollout through create_hidden_state_root /
    evaluate_state / hidden_state_transition, loss_fn, loss.backward(), optimizer.step() — on the reference's two
    training minibatches (tests/golden/learner_small.npz, narrow nets). The three nets run on the device learner's
    HIP kernels behind torch.autograd. Against the reference: both steps' losses and logits within rtol 2e-4, the
    parameters after each Adam step within 2 lr (first-step updates are ~lr sign(g)), BN running statistics rtol
    1e-4. Against mzba.learner.Learner.train_minibatch on the same minibatch (same kernels, its fused loss kernel):
    gradients within 1e-4 of each tensor's magnitude. Then eval_mode() puts the trained weights into the packed
    inference nets (the target-net copy, train_torch.py:361-367, reads them through state_dict()), and the
    optimizer's state_dict is torch.optim.Adam's (train_torch.py:622, 652) and round-trips."""
    import os
    from conftest import GOLDEN
    from mzba.config import learner_model_cfg
    from mzba.learner import Learner, MinibatchRing
    from mzba.weights import init_state_dict
    from src.networks import MuZeroAgent
    from utils import ScalarTransforms
    z = np.load(os.path.join(GOLDEN, "learner_small.npz"))
    mcfg, K, lr = learner_model_cfg(), int(z["K"]), float(z["lr"])
    mcfg = dict(mcfg, learning_rate=lr, device="cuda", dtype="f32")  # narrow nets: the f32 inference path
    start = init_state_dict(mcfg, int(z["seed"]))
    ag = MuZeroAgent(mcfg)
    ag.load_state_dict(start)
    st = ScalarTransforms(mcfg)
    ref_ln = Learner(mcfg, start, K=K, streams=1, defer_wgrad=False)
    ag.train_mode()
    for s in (1, 2):
        mb = {k.split("/")[-1]: z[k] for k in z.files if k.startswith(f"s{s}/in/")}
        loss, logits = _training_iteration(ag, st, mb, K, mcfg["state_history_length"], mcfg["latent_resolution"])
        ref = np.array([float(z[f"s{s}/{k}"]) for k in ("loss", "rl", "vl", "pl")])
        np.testing.assert_allclose(loss, ref, rtol=2e-4, atol=2e-5, err_msg=f"step {s} losses")
        for got, key in zip(logits, ("pr", "pv", "pp")):
            np.testing.assert_allclose(got.cpu().numpy(), z[f"s{s}/{key}"], rtol=2e-4, atol=5e-5, err_msg=f"step {s} {key}")
        # the same minibatch through the learner's own fused minibatch (its loss kernel), from the same state
        ring = MinibatchRing(mb)
        ref_ln.train_minibatch(ring, ring.slots())
        g_ref, g_got = ref_ln.gradients(), ag._learner.gradients()
        for k, g in g_ref.items():
            a, b = g.numpy().astype(np.float64), g_got[k].numpy().astype(np.float64)
            scale = max(np.abs(a).max(), 1e-30)
            if k.endswith((".conv1.bias", ".conv2.bias", ".conv.bias")):  # pre-BN biases: exactly 0 up to rounding
                continue
            assert np.abs(a - b).max() <= 1e-4 * scale + 1e-9, (s, k, np.abs(a - b).max() / scale)
        sd = ag.state_dict()
        for k, v in sd.items():
            want = z[f"s{s}/param/{k}"].astype(np.float64)
            got = v.numpy().astype(np.float64)
            if k.endswith(("running_mean", "running_var")):
                np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-6, err_msg=k)
            elif k.endswith("num_batches_tracked"):
                assert int(got) == int(want), k
            else:
                assert np.abs(got - want).max() <= 2.0 * lr * 1.001, (s, k, np.abs(got - want).max() / lr)
        # teacher forcing for step 2, as the learner test: the reference's post-step-1 state
        if s == 1:
            nxt = {k[len("s1/param/"):]: z[k] for k in z.files if k.startswith("s1/param/")}
            opt = {"state": {i: {"step": torch.tensor(1.0), "exp_avg": torch.as_tensor(z[f"s1/opt/exp_avg/{k}"]),
                                 "exp_avg_sq": torch.as_tensor(z[f"s1/opt/exp_avg_sq/{k}"])}
                             for i, k in enumerate(ref_ln.params)},
                   "param_groups": ag.optimizer.state_dict()["param_groups"]}
            ag.load_state_dict(nxt)          # train_torch.py:645-652: model, then optimizer
            ag.optimizer.load_state_dict(opt)
            ref_ln.load_state_dict(nxt)
            ref_ln.load_optimizer_state_dict(opt)
    # the optimizer state round-trips in torch.optim.Adam's format
    osd = ag.optimizer.state_dict()
    assert len(osd["state"]) == len(list(ag.parameters())) and float(osd["state"][0]["step"]) == 2.0
    adam = torch.optim.Adam([torch.zeros_like(p) for p in ag.parameters()], lr=lr, weight_decay=1e-4)
    adam.load_state_dict(osd)
    # eval_mode: the host copy holds the trained weights and running statistics (what the target-net copy,
    # train_torch.py:361-367, reads through state_dict()); these 32-channel nets have no packed inference form
    # (PackedNets needs multiples of 64 channels), so the pack refresh is checked on the 64-channel nets below
    trained = {k: v.clone() for k, v in ag.state_dict().items()}
    ag.eval_mode()
    for k, v in ag.state_dict().items():
        assert torch.equal(v, trained[k]), k


def test_dropin_agent_eval_after_training_refreshes_the_packed_nets():
    """A 64-channel agent whose packed inference nets exist (acting) trains one reference minibatch body in
    train_mode() (synthetic replay windows), then eval_mode(): its packed nets equal, tensor for tensor, a fresh
    agent's built from the trained state_dict (BN folded from the trained running statistics), and its inference
    matches the numpy oracle of those weights within 1e-5 (f32 path)."""
    from mzba.config import small_model_cfg
    from mzba.weights import init_state_dict
    from oracle import nets as N
    from src.networks import MuZeroAgent
    from utils import ScalarTransforms
    mcfg = dict(small_model_cfg(default_config()), device="cuda", dtype="f32")
    ag = MuZeroAgent(mcfg)
    ag.load_state_dict(init_state_dict(mcfg, 3))
    x = torch.rand(5, 2 * mcfg["state_history_length"], 16, 20, device="cuda")
    h0 = ag.create_hidden_state_root(x)  # the packed nets exist before training
    g = np.random.default_rng(4)
    B, K, Lh = 6, 5, mcfg["state_history_length"]
    lut = np.array([0, 0.3, 0.6, 1.0], np.float32)
    mb = dict(states=lut[g.integers(0, 4, (B, Lh, 16, 20))], past_actions=g.integers(0, 3, (B, Lh)),
              future_actions=g.integers(0, 3, (B, K)), rewards=g.choice(np.array([-1, 0, 1], np.float32), (B, K)),
              targets=(g.normal(size=(B, K)) * 2).astype(np.float32),
              counts=g.multinomial(50, [0.3, 0.3, 0.4], (B, K)).astype(np.float32) + 1)
    ag.train_mode()
    loss, _ = _training_iteration(ag, ScalarTransforms(mcfg), mb, K, Lh, mcfg["latent_resolution"])
    assert np.isfinite(loss).all()
    ag.eval_mode()
    trained = ag.state_dict()
    ref = MuZeroAgent(mcfg)
    ref.load_state_dict(trained)
    for a, b in zip(ag.packed.device_tensors(), ref.packed.device_tensors()):
        assert torch.equal(a, b)
    got = ag.create_hidden_state_root(x)
    assert not torch.equal(got, h0)  # the weights moved
    want = N.create_hidden_state_root(x.cpu().numpy(), {k: v.numpy() for k, v in trained.items()}, mcfg)
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-5, atol=1e-5)
