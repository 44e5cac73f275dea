"""Command-line surface.

``train_parser()`` keeps every flag and default of the reference ``train.py`` (train.py:15-69,
SURVEY.md §5.6) and adds MI355X-era flags.  ``sample_parser()`` mirrors sample.py:13-23 and
``splitter_parser()`` mirrors data_splitter.py:9-12.  Unlike the reference, nothing is parsed at
import time, so the entry points are importable as a library.
"""
from __future__ import annotations

import argparse


def train_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                description="Train a character-level RNN language model on "
                                            "AMD MI355X (gfx950) or CPU.")
    # --- reference flags (train.py:17-69) ---------------------------------------------
    p.add_argument("--data_dir", type=str, default="data/tinyshakespeare",
                   help="data directory containing input.txt with training examples")
    p.add_argument("--save_dir", type=str, default="save",
                   help="directory to store checkpointed models")
    p.add_argument("--log_dir", type=str, default="logs",
                   help="directory to store tensorboard-compatible event logs and metrics")
    p.add_argument("--save_every", type=int, default=1000,
                   help="Save frequency. Number of passes between checkpoints of the model.")
    p.add_argument("--init_from", type=str, default=None,
                   help="continue training from saved model at this path. The path must "
                        "contain config.pkl, chars_vocab.pkl, checkpoint and model.ckpt-* "
                        "files; model, rnn_size, num_layers and seq_length must match.")
    p.add_argument("--model", type=str, default="lstm", help="lstm, rnn, gru, or nas")
    p.add_argument("--rnn_size", type=int, default=128, help="size of RNN hidden state")
    p.add_argument("--num_layers", type=int, default=2, help="number of layers in the RNN")
    p.add_argument("--seq_length", type=int, default=50,
                   help="RNN sequence length. Number of timesteps to unroll for.")
    p.add_argument("--batch_size", type=int, default=50,
                   help="minibatch size per worker (sequences propagated in parallel)")
    p.add_argument("--num_epochs", type=int, default=50, help="number of epochs")
    p.add_argument("--grad_clip", type=float, default=5.0, help="clip gradients at this global norm")
    p.add_argument("--clip_norm", choices=["tf", "dense"], default="tf",
                   help="embedding term of the clip norm: 'tf' = per-token IndexedSlices values "
                        "(TF 1.x, the reference), 'dense' = the summed [V, H] gradient")
    p.add_argument("--learning_rate", type=float, default=0.002, help="learning rate")
    p.add_argument("--decay_rate", type=float, default=0.97,
                   help="per-epoch exponential learning-rate decay (Adam)")
    p.add_argument("--output_keep_prob", type=float, default=1.0,
                   help="probability of keeping weights in the hidden layer")
    p.add_argument("--input_keep_prob", type=float, default=1.0,
                   help="probability of keeping weights in the input layer")
    p.add_argument("--distributed", action="store_true", help="Indicates running in distributed mode")
    p.add_argument("--ps_hosts", default=None,
                   help="PS HOSTS (host:port). The ps process hosts the rendezvous store")
    p.add_argument("--worker_hosts", default=None, help="WORKER HOSTS (comma-separated host:port)")
    p.add_argument("--job_name", choices=["ps", "worker"], default=None,
                   help="Job name. Must be ps/worker")
    p.add_argument("--task_index", type=int, default=None, help="Index of task for given job")
    p.add_argument("--tensor_file", default=None,
                   help="Tensor file of the specific training data for given node")
    # --- MI355X-era additions -----------------------------------------------------------
    g = p.add_argument_group("framework")
    g.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"],
                   help="execution device (auto = GPU when available)")
    g.add_argument("--dtype", default="auto", choices=["auto", "bf16", "fp32"],
                   help="compute dtype (auto = bf16 on GPU, fp32 on CPU).  The native HIP kernels "
                        "compute with bf16 MFMA operands (fp32 state and accumulation); fp32 on a "
                        "GPU runs every LSTM / GRU / RNN cell step on the fp32-operand kernels "
                        "(csrc/cell_f32.hip, a numerics mode; NAS: the autograd path)")
    g.add_argument("--seed", type=int, default=0, help="parameter-init / dropout seed")
    g.add_argument("--log_every", type=int, default=1, help="print a progress line every N steps")
    g.add_argument("--summary_every", type=int, default=100,
                   help="write logits/loss histograms to the event log every N steps (0 = off)")
    g.add_argument("--metrics_file", default=None,
                   help="JSONL metrics stream (default: <log_dir>/<run>/metrics.jsonl)")
    g.add_argument("--bucket_mb", type=float, default=8.0,
                   help="gradient all-reduce bucket size in MB (data parallel)")
    g.add_argument("--allreduce_dtype", default="fp32", choices=["fp32", "bf16"],
                   help="wire dtype of the gradient exchange (bf16 with --dp_mode sharded: "
                        "fp32 accumulation on the receiving rank)")
    g.add_argument("--dp_mode", default="replicated", choices=["replicated", "sharded"],
                   help="replicated: bucketed all-reduce + every rank updates every parameter; "
                        "sharded: reduce-scatter + clip/Adam on this rank's 1/world shard + "
                        "all-gather (ZeRO stage 1, parallel/zero.py)")
    g.add_argument("--dist_backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="torch.distributed backend (nccl = RCCL on ROCm)")
    g.add_argument("--dist_timeout", type=float, default=600.0,
                   help="collective timeout in seconds (failure detection)")
    g.add_argument("--synthetic_text", type=int, default=0,
                   help="train on N chars of Shakespeare-shaped synthetic text instead of data_dir")
    g.add_argument("--max_steps", type=int, default=0, help="stop after N steps (0 = no limit)")
    g.add_argument("--resume_exact", action="store_true",
                   help="with --init_from, continue from the saved epoch/batch instead of "
                        "restarting the epoch counter (reference behaviour)")
    g.add_argument("--save_state", action="store_true",
                   help="also checkpoint the TBPTT carry state")
    g.add_argument("--profile", action="store_true",
                   help="emit roctx ranges per phase and print a per-phase timing table")
    g.add_argument("--heartbeat", type=float, default=0.0,
                   help="seconds between rank heartbeats in the rendezvous store (0 = off)")
    g.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                   help="replay the whole GPU training step (forward, BPTT, weight gradients, "
                        "clip + Adam) as one captured HIP graph (engine/graph_step.py); auto = "
                        "on wherever it applies (one rank, native backend, no dropout) for "
                        "launch-bound steps (B·T·rnn_size <= 2^21)")
    return p


def sample_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--save_dir", type=str, default="save",
                   help="model directory to store checkpointed models")
    p.add_argument("-n", type=int, default=500, help="number of characters to sample")
    p.add_argument("--prime", type=str, default="", help="prime text")
    p.add_argument("--sample", type=int, default=1,
                   help="0 to use max at each timestep, 1 to sample at each timestep, "
                        "2 to sample on spaces")
    p.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    p.add_argument("--seed", type=int, default=None, help="sampling RNG seed")
    p.add_argument("--num_samples", type=int, default=1,
                   help="independent samples drawn in parallel (batched on the device)")
    p.add_argument("--bytes", action="store_true",
                   help="print the utf-8 bytes repr like the reference did on python 3 (A-15)")
    return p


def splitter_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", help="Data directory containing the dataset.", required=True)
    p.add_argument("--num_parts", type=int, required=True,
                   help="Number of parts in which to divide, same as amount of worker nodes")
    p.add_argument("--out_dir", default="sharded_data",
                   help="Output directory. Will contain files as 'data-<num>.npy'")
    p.add_argument("--exact", action="store_true",
                   help="require an exact split like the reference np.split (errors otherwise)")
    return p
