"""Default configuration: the values of the reference's `config.yaml` (`parameters:`,
config.yaml:1-61), as a dict with the same schema so the reference's YAML loads
into every class here unchanged (`yaml.safe_load(f)["parameters"]`).

Values the reference overrides in code are noted where they are applied:
env H/W/brick rows (parallel_breakout.py:76-79), Dirichlet alpha/weight
(mcts.py:21-22), temperature schedule (train_torch.py:82,129-135).
"""
import copy

_DEFAULT = {
    "num_iterations": 50000,
    "num_episodes": 2,
    "num_unroll_steps": 5,
    "num_simulations": 50,
    "actions": [0, 1, 2],
    "minibatch_size": 512,
    "num_batches": 15,
    "discount_factor": 0.985,
    "latent_resolution": [4, 5],
    "real_resolution": [16, 20],
    "n_parallel": 24,
    "samples_before_train": 35000,
    "replay_buffer_max": 60000,
    "load_weights": False,
    "checkpoint_path": "weights/checkpt1.pth",
    "search": {"mcts_name": "MCTSSearchVec", "c1": 1.25, "c2": 19652.0, "discount_factor": 0.985},
    "model": {
        "learning_rate": 0.0002,
        "agent_name": "MuZeroAgent",
        "num_supports": 11,
        "supports_min": -5,
        "supports_max": 5,
        "latent_channels": [128, 256],
        "state_history_length": 32,
        "device": "cuda",
        "latent_resolution": [4, 5],
        "representation_network": {"num_res_blocks": [2, 3, 3], "activation": "relu"},
        "dynamics_network": {"num_res_blocks": 14, "num_actions": 3, "activation": "relu"},
        "prediction_network": {"num_res_blocks": 14, "num_actions": 3, "activation": "relu"},
    },
    "environment": {
        "environment_name": "BreakoutEnvironment",
        "environment_path": "environment.parallel_breakout",
        "resolution": [16, 16],
        "brick_rows": 5,
        "n_parallel": 24,
        "paddle_hit_reward": 0.0,
        "brick_hit_reward": 1.0,
        "game_lost_reward": -1.0,
        "game_won_reward": 5.0,
    },
}


def default_config():
    return copy.deepcopy(_DEFAULT)


def small_model_cfg(cfg=None):
    """Reduced-width model used by the fast parity fixtures (tests/golden)."""
    cfg = cfg or default_config()
    m = copy.deepcopy(cfg["model"])
    m["latent_channels"] = [64, 64]
    m["state_history_length"] = 4
    m["representation_network"] = {"num_res_blocks": [1, 1, 1], "activation": "relu"}
    m["dynamics_network"] = {"num_res_blocks": 2, "num_actions": 3, "activation": "relu"}
    m["prediction_network"] = {"num_res_blocks": 2, "num_actions": 3, "activation": "relu"}
    m["device"] = "cpu"
    return m


def learner_model_cfg(cfg=None):
    """The narrow learner fixture config (tests/golden/learner_small.npz): 32 channels, L = 4."""
    m = small_model_cfg(cfg)
    m["latent_channels"] = [32, 32]
    return m
