"""Drop-in for the reference CLI runners/torch_run_physics.py (:1-117).

Same flags, names, types, defaults and store_true/store_false semantics
(:10-34), same task table (:49-75), same train-then-test flow (:77-117);
the model is the HIP-backed PhysicsNet of this package.

Additive flags only:
  --loss_mode {fresh,reference}  fresh (default): the loss is the current
        forward's; reference: reproduce quirk Q1 (stale self.output).
  --data_dir DIR                 where <task file> lives (default: the
        reference's data/datasets relative to this runner, :86-89).
  --synthetic N                  if the task's npz is missing, render one with
        N training sequences (N//10 valid/test) with nn/datasets/synth.py.
  --seed S                       shared shuffle seed (required for DDP sharding).
  --device_data {1,0}            1 (default): uint8 dataset resident in HBM, each
        batch gathered on the GPU; 0: the reference's host path.

Data-parallel training: launch with torchrun (one process per GPU, RCCL);
--batch_size is per rank, every rank draws a disjoint shard of each epoch.

    PYTHONPATH=. python runners/torch_run_physics.py --task spring_color --color \\
        --autoencoder_loss 3.0 --save_dir /tmp/run --synthetic 2000
"""
import argparse
import logging
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.abspath(os.path.join(os.path.dirname(os.path.realpath(__file__)), ".."))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from paig_reproduction_amd.nn.network import physics_models  # noqa: E402
from paig_reproduction_amd.nn.utils.misc import classes_in_module  # noqa: E402
from paig_reproduction_amd.nn.datasets.iterators import get_iterators  # noqa: E402

TASKS = {
    # task: (train file, test file, cell, seq_len, test_seq_len, input_steps, pred_steps, input_size)
    "bouncing_balls": ("bouncing/color_bounce_vx8_vy8_sl12_r2.npz", "bouncing/color_bounce_vx8_vy8_sl30_r2.npz",
                       "bouncing_ode_cell", 12, 30, 4, 6, 32 * 32),
    "spring_color": ("spring_color/color_spring_vx8_vy8_sl12_r2_k4_e6.npz",
                     "spring_color/color_spring_vx8_vy8_sl30_r2_k4_e6.npz", "spring_ode_cell", 12, 30, 4, 6, 32 * 32),
    "spring_color_half": ("spring_color_half/color_spring_vx4_vy4_sl12_r2_k4_e6_halfpane.npz",
                          "spring_color_half/color_spring_vx4_vy4_sl30_r2_k4_e6_halfpane.npz", "spring_ode_cell",
                          12, 30, 4, 6, 32 * 32),
    "3bp_color": ("3bp_color/color_3bp_vx2_vy2_sl20_r2_g60_m1_dt05.npz",
                  "3bp_color/color_3bp_vx2_vy2_sl40_r2_g60_m1_dt05.npz", "gravity_ode_cell", 20, 40, 4, 12, 36 * 36),
    "mnist_spring_color": ("mnist_spring_color/color_mnist_spring_vx8_vy8_sl12_r2_k2_e12.npz",
                           "mnist_spring_color/color_mnist_spring_vx8_vy8_sl30_r2_k2_e12.npz", "spring_ode_cell",
                           12, 30, 3, 7, 64 * 64),
}


def build_parser():
    p = argparse.ArgumentParser(description="PyTorch version of the TensorFlow script.")
    p.add_argument("--epochs", type=int, default=10, help="Number of epochs to train")
    p.add_argument("--batch_size", type=int, default=100, help="Training batch size (per rank)")
    p.add_argument("--save_dir", type=str, default="", help="Directory to save checkpoint and logs")
    p.add_argument("--use_ckpt", action="store_true", help="Whether to start from scratch or start from checkpoint")
    p.add_argument("--ckpt_dir", type=str, default="", help="Checkpoint directory to use")
    p.add_argument("--base_lr", type=float, default=1e-3, help="Base learning rate")
    p.add_argument("--anneal_lr", action="store_false", help="Whether to anneal lr after 0.75 of total epochs")
    p.add_argument("--optimizer", type=str, default="rmsprop", help="Optimizer to use")
    p.add_argument("--save_every_n_epochs", type=int, default=5, help="Epochs between checkpoint saves")
    p.add_argument("--eval_every_n_epochs", type=int, default=1, help="Epochs between validation run")
    p.add_argument("--print_interval", type=int, default=10, help="Print train metrics every n mini-batches")
    p.add_argument("--debug", action="store_true", help="If true, eval is not run before training")
    p.add_argument("--test_mode", action="store_true", help="If true, only run test set")
    p.add_argument("--task", type=str, default="", help="Type of task.")
    p.add_argument("--model", type=str, default="PhysicsNet", help="Model to use.")
    p.add_argument("--recurrent_units", type=int, default=100,
                   help="Number of units for each lstm, if using black-box dynamics.")
    p.add_argument("--lstm_layers", type=int, default=1,
                   help="Number of lstm cells to use, if using black-box dynamics")
    p.add_argument("--cell_type", type=str, default="", help="Type of pendulum to use.")
    p.add_argument("--encoder_type", type=str, default="conv_encoder", help="Type of encoder to use.")
    p.add_argument("--decoder_type", type=str, default="conv_st_decoder", help="Type of decoder to use.")
    p.add_argument("--autoencoder_loss", type=float, default=0.0, help="Autoencoder loss weighing.")
    p.add_argument("--alt_vel", action="store_true", help="Whether to use linear velocity computation.")
    p.add_argument("--color", action="store_true", help="Whether images are RGB or grayscale.")
    p.add_argument("--datapoints", type=int, default=0,
                   help="How many datapoints from the dataset to use. Default=0 uses all data.")
    # additive
    p.add_argument("--loss_mode", choices=("fresh", "reference"), default="fresh")
    p.add_argument("--data_dir", type=str, default=os.path.join(REPO, "data", "datasets"))
    p.add_argument("--synthetic", type=int, default=0)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                   help="fp32: fp32-accurate results (convs/GEMMs on the 16-bit matrix cores with split "
                        "hi+lo operands); bf16: bf16 operands, fp32 accumulation (BASELINE config #2)")
    p.add_argument("--conv_math", choices=("split", "fp32", "bf16"), default=None,
                   help="override the conv/GEMM arithmetic directly (fp32 = f32-input MFMA)")
    p.add_argument("--device_data", type=int, default=1,
                   help="1: dataset resident in HBM as uint8, batches gathered on the GPU (F2); 0: host iterators")
    return p


def dataset_path(args, rel, seq_len):
    path = os.path.join(args.data_dir, rel)
    if not os.path.exists(path) and args.synthetic > 0:
        from paig_reproduction_amd.nn.datasets.synth import write_dataset
        if _rank() == 0:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            n = args.synthetic
            write_dataset(path, args.task, seq_len, n, max(n // 10, 1), max(n // 10, 1), seed=0)
        if dist.is_initialized():
            dist.barrier()
    return path


def _rank():
    return dist.get_rank() if dist.is_initialized() else 0


def main(argv=None):
    args = build_parser().parse_args(argv)
    logger = logging.getLogger("torch")
    logger.setLevel(logging.DEBUG)
    if not logger.handlers:
        ch = logging.StreamHandler()
        ch.setLevel(logging.DEBUG)
        ch.setFormatter(logging.Formatter('%(asctime)s - %(name)s - %(message)s'))
        logger.addHandler(ch)

    Model = classes_in_module(physics_models)[args.model]
    data_file, test_data_file, cell_type, seq_len, test_seq_len, input_steps, pred_steps, input_size = \
        TASKS[args.task]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("paig_reproduction_amd trains on the GPU only (HIP kernels); no CUDA/ROCm device found")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        if args.seed is None:
            args.seed = 0   # every rank must shuffle with the same permutation
    device = torch.device(f"cuda:{local}")
    rank = _rank()

    def make(sl):
        if args.seed is not None:
            torch.manual_seed(args.seed)
        net = Model(args.task, args.recurrent_units, args.lstm_layers, cell_type, sl, input_steps, pred_steps,
                    args.autoencoder_loss, args.alt_vel, args.color, input_size, args.encoder_type,
                    args.decoder_type, device=device)
        net.loss_mode = args.loss_mode
        net.conv_math = args.conv_math or ("bf16" if args.dtype == "bf16" else "split")
        net.to(net.device)
        if world > 1:
            for t in net.state_dict().values():
                dist.broadcast(t, 0)
        return net

    if not args.test_mode:
        network = make(seq_len)
        its = get_iterators(dataset_path(args, data_file, seq_len), conv=True, datapoints=args.datapoints,
                            seed=args.seed, rank=rank, world=world, device=device if args.device_data else None)
        network.get_data(its)
        network.build_optimizer(args.base_lr, args.optimizer, args.anneal_lr)
        network.initialize_graph(args.save_dir, args.use_ckpt, args.ckpt_dir)
        network.train_model(args.epochs, args.batch_size, args.save_every_n_epochs, args.eval_every_n_epochs,
                            args.print_interval, args.debug)

    network = make(test_seq_len)
    network.build_optimizer(args.base_lr, args.optimizer, args.anneal_lr)
    network.initialize_graph(args.save_dir, True, args.ckpt_dir)
    its = get_iterators(dataset_path(args, test_data_file, test_seq_len), conv=True, datapoints=args.datapoints,
                        seed=args.seed, rank=rank, world=world, device=device if args.device_data else None)
    network.get_data(its)
    network.train_model(0, args.batch_size, args.save_every_n_epochs, args.eval_every_n_epochs,
                        args.print_interval, args.debug)
    if world > 1:
        dist.destroy_process_group()
    return network


if __name__ == "__main__":
    main()
