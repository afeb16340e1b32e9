"""runners/torch_run_physics.py: the reference CLI surface (flags, defaults,
store_true/store_false semantics of runners/torch_run_physics.py:10-34) and a
tiny end-to-end train -> checkpoint -> test run on the GPU."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(REPO, "runners"))

# (flag, default) of the reference parser, runners/torch_run_physics.py:10-34
REFERENCE_FLAGS = {
    "epochs": 10, "batch_size": 100, "save_dir": "", "use_ckpt": False, "ckpt_dir": "", "base_lr": 1e-3,
    "anneal_lr": True, "optimizer": "rmsprop", "save_every_n_epochs": 5, "eval_every_n_epochs": 1,
    "print_interval": 10, "debug": False, "test_mode": False, "task": "", "model": "PhysicsNet",
    "recurrent_units": 100, "lstm_layers": 1, "cell_type": "", "encoder_type": "conv_encoder",
    "decoder_type": "conv_st_decoder", "autoencoder_loss": 0.0, "alt_vel": False, "color": False, "datapoints": 0,
}


def test_cli_flags_match_reference():
    import torch_run_physics as R
    ns = R.build_parser().parse_args([])
    for k, v in REFERENCE_FLAGS.items():
        assert getattr(ns, k) == v, k
    ns = R.build_parser().parse_args(["--anneal_lr", "--use_ckpt", "--alt_vel", "--color", "--debug"])
    assert ns.anneal_lr is False and ns.use_ckpt and ns.alt_vel and ns.color and ns.debug
    assert ns.loss_mode == "fresh"
    assert set(R.TASKS) == {"bouncing_balls", "spring_color", "spring_color_half", "3bp_color", "mnist_spring_color"}
    assert R.TASKS["3bp_color"][2:] == ("gravity_ode_cell", 20, 40, 4, 12, 36 * 36)
    assert R.TASKS["mnist_spring_color"][2:] == ("spring_ode_cell", 12, 30, 3, 7, 64 * 64)


@pytest.fixture
def torch_logger():
    import logging
    lg = logging.getLogger("torch")     # the reference logs to the "torch" logger (runner :38-44)
    handlers, level = list(lg.handlers), lg.level
    yield lg
    for h in list(lg.handlers):
        if h not in handlers:
            lg.removeHandler(h)
    lg.setLevel(level)


@pytest.mark.gpu
def test_cli_train_then_test(tmp_path, torch_logger):
    import torch_run_physics as R
    save = str(tmp_path / "run")
    data = str(tmp_path / "data")
    net = R.main(["--task", "spring_color", "--color", "--autoencoder_loss", "3.0", "--epochs", "2",
                  "--batch_size", "10", "--save_dir", save, "--save_every_n_epochs", "1", "--print_interval", "1",
                  "--data_dir", data, "--synthetic", "40", "--seed", "0"])
    assert os.path.exists(os.path.join(save, "model.ckpt"))
    assert os.path.exists(os.path.join(save, "outputs.npz"))
    out = np.load(os.path.join(save, "outputs.npz"))
    assert out["input"].shape[1:] == (30, 3, 32, 32)           # test_seq_len
    assert np.isfinite(out["output"]).all()
    assert net.output.shape[1] == 30 - 4                      # test-mode rollout length
