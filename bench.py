#!/usr/bin/env python
"""Headline benchmark: whole-node training throughput (chars/sec) of the 2-layer LSTM-512,
seq 128, vocab 65 char-RNN (BASELINE.json), bf16, synthetic Shakespeare-shaped text,
random-init weights, synchronous data parallel over RCCL (one process per GPU).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Each timed step is a complete training step of the framework: device batch of token ids ->
forward (fused HIP recurrent kernels) -> fused softmax-CE -> BPTT -> bucketed gradient
all-reduce (RCCL) -> fused global-norm clip + TF-Adam -> weights refreshed for the next step,
with the TBPTT state carried across steps as in train.py.  Per-GPU batch is fixed as N grows
(weak scaling).  Rank 0 prints ONE JSON line; the time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch
import torch.distributed as dist

METRIC = "chars/sec (whole node), 2-layer LSTM-512 seq128, at 1/2/4/8 MI355X"
MIOPEN_1GPU_CPS = 2098017.9  # torch.nn.LSTM (MIOpen) bf16, B=256, same config, 1x MI355X
                             # (scripts/bench_miopen_lstm.py)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (sequences)")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--vocab", type=int, default=65)
    ap.add_argument("--model", default="lstm")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype on the GPU: bf16 MFMA operands (default) or the native "
                         "fp32-operand recurrence (engine/native/fp32.py, a numerics mode)")
    ap.add_argument("--bucket_mb", type=float, default=8.0)
    ap.add_argument("--allreduce_dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--dp_mode", default="replicated", choices=["replicated", "sharded"],
                    help="sharded: reduce-scatter + Adam on a 1/world shard + all-gather")
    ap.add_argument("--clip_norm", default="tf", choices=["tf", "dense"],
                    help="embedding term of the clip norm (default: TF per-token semantics)")
    ap.add_argument("--input_keep_prob", type=float, default=1.0,
                    help="dropout (DropoutWrapper input keep prob; default off as in the reference)")
    ap.add_argument("--output_keep_prob", type=float, default=1.0,
                    help="dropout (DropoutWrapper output + embedding keep prob)")
    ap.add_argument("--profile", action="store_true",
                    help="print a per-phase timing table and the gradient buckets' overlap windows")
    ap.add_argument("--force_sync", action="store_true",
                    help="run the bucketed RCCL gradient exchange even on one rank (measures its "
                         "cost and release schedule on a one-GPU box)")
    ap.add_argument("--graph", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="replay each step from one captured HIP graph (one GPU, no dropout); "
                         "auto (the default, as train.py) = only for launch-bound steps "
                         "(batch x seq x hidden <= 2^21), where the replay wins; eager otherwise")
    ap.add_argument("--dist_backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto = nccl (RCCL over xGMI) on GPUs; gloo = multi-rank rehearsal on "
                         "one GPU (with DCR_RECURRENCE=step: persistent grids of two processes cannot "
                         "share the CUs)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = plumbing check of the multi-rank contract (reference backend, gloo)")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = parse(argv)
    from distributed_char_rnn_amd.engine.optim import TFAdam
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig
    from distributed_char_rnn_amd.parallel import process_group, topology
    from distributed_char_rnn_amd.parallel.grad_sync import GradSync
    from distributed_char_rnn_amd.utils.data import synthetic_tokens

    topo = topology.from_env() or topology.Topology()
    if topo.world_size != a.gpus:
        if a.gpus > 1 and topo.world_size == 1:
            print(f"--gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes",
                  file=sys.stderr)
            return 2
    device = process_group.pick_device(topo, a.device)
    backend = a.dist_backend if a.dist_backend != "auto" else (
        "nccl" if device.type == "cuda" else "gloo")
    ctx = process_group.init(topo, device, backend)

    def sync_dev():
        if device.type == "cuda":
            torch.cuda.synchronize()
    rank, world = max(ctx.rank, 0), ctx.world_size

    cfg = ModelConfig(model=a.model, vocab_size=a.vocab, rnn_size=a.hidden, num_layers=a.layers,
                      clip_norm=a.clip_norm, input_keep_prob=a.input_keep_prob,
                      output_keep_prob=a.output_keep_prob)
    model = CharRNN(cfg, device=device, seed=1234, dtype=a.dtype)
    opt = TFAdam(model.store, clip=5.0, guard=model.error_word())
    model.bind_optimizer(opt)  # fused Adam + weight layouts (csrc/tail.hip)
    # (--force_sync: the exchange also runs on one rank, sharded or replicated)
    sharded = a.dp_mode == "sharded" and (world > 1 or a.force_sync)
    sync = GradSync(model.store, world, a.bucket_mb, a.allreduce_dtype,
                    enabled=(world > 1 or a.force_sync) and not sharded,
                    guard=model.error_word(), timing=a.profile)
    if (a.force_sync or sharded) and a.graph == "on":
        # the captured step never calls sync.ready, so nothing would write the guard slot and
        # the exchange would not be measured at all
        raise SystemExit("bench.py: --force_sync measures the eager bucketed exchange; "
                         "drop --graph")
    if sync.enabled and sync.guard_view is not None:
        opt.guard = sync.guard_view  # every rank's error word, summed with the last bucket
    if a.force_sync and world == 1 and not dist.is_initialized():
        import os

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group(backend, rank=0, world_size=1)
    if world > 1:
        dist.broadcast(model.store.flat, 0)
    zstep = None
    if sharded:
        from distributed_char_rnn_amd.parallel.zero import ShardedStep

        zstep = ShardedStep(model.store, opt, world, rank, wire=a.allreduce_dtype,
                            bucket_mb=a.bucket_mb, guard=model.error_word())
    model.params_changed()

    B, T = a.batch, a.seq
    nbat = 16
    toks = synthetic_tokens(nbat * B * T + 1, a.vocab, seed=1000 + rank)
    data = torch.from_numpy(toks).to(device)
    xs = data[:-1].view(B, nbat * T)          # row-contiguous streams like TextLoader
    ys = data[1:].view(B, nbat * T)
    state = model.zero_state(B)
    prof = None
    if a.profile:
        from distributed_char_rnn_amd.utils.metrics import PhaseProfiler

        prof = PhaseProfiler(True, device)

    graphed = None
    use_graph = a.graph == "on"
    if a.graph == "auto":
        from distributed_char_rnn_amd.engine.trainer import GRAPH_AUTO_MAX_WORK

        use_graph = (not (a.force_sync or sharded) and torch.device(device).type == "cuda"
                     and B * T * a.hidden <= GRAPH_AUTO_MAX_WORK)
    if use_graph:
        from distributed_char_rnn_amd.engine.graph_step import GraphedStep

        ok, why = GraphedStep.supported(model, world)
        if not ok and a.graph == "on":
            print(f"--graph: {why}", file=sys.stderr)
            return 2
        if ok:
            graphed = GraphedStep(model, opt, log=lambda m: print(m, file=sys.stderr))

    def step(i, state):
        k = i % nbat
        x = xs[:, k * T:(k + 1) * T]
        y = ys[:, k * T:(k + 1) * T]
        if k == 0:
            state = model.zero_state(B)
        if graphed is not None:
            return graphed(x, y, state, 2e-3)
        if zstep is not None:  # each bucket's reduce-scatter leaves during the backward
            zstep.reset()
            if prof is None:
                loss, state, _ = model.train_step(x, y, state, zstep)
                zstep.step(2e-3)
            else:
                with prof.phase("fwd_bwd"):
                    loss, state, _ = model.train_step(x, y, state, zstep)
                with prof.phase("sharded_step"):
                    zstep.step(2e-3)
            return loss, state
        sync.reset()
        if prof is None:
            loss, state, _ = model.train_step(x, y, state, sync)
            gs = sync.finish(defer_scale=True)
            opt.step(2e-3, grad_scale=gs)
        else:
            with prof.phase("fwd_bwd"):
                loss, state, _ = model.train_step(x, y, state, sync)
            with prof.phase("grad_sync"):
                gs = sync.finish(defer_scale=True)
            with prof.phase("optimizer"):
                opt.step(2e-3, grad_scale=gs)
        return loss, state

    for i in range(a.warmup):
        loss, state = step(i, state)
    sync_dev()
    if prof is not None:
        prof.collect()
        prof.totals.clear()
        prof.counts.clear()
    ctx.barrier()
    sync_dev()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss, state = step(a.warmup + i, state)
    ctx.barrier()
    sync_dev()
    dt = time.perf_counter() - t0
    dt = ctx.all_reduce_scalar(dt, dist.ReduceOp.MAX) if world > 1 else dt
    final_loss = float(loss)
    check = getattr(model.backend, "check_errors", None)
    if check is not None:  # a persistent kernel that timed out would have produced garbage
        check()
    ms = dt / a.steps * 1e3
    cps = world * B * T * a.steps / dt
    if rank == 0:
        if prof is not None:
            print(prof.table(), file=sys.stderr)
            if zstep is not None:
                print(f"sharded: {zstep.early} of {len(zstep.buckets)} bucket "
                      f"reduce-scatters launched during the backward (last step)", file=sys.stderr)
            win = sync.windows()
            if win:
                print("gradient buckets (last step): release after step start / overlap window "
                      "until the backward ends", file=sys.stderr)
                for i, nb, t, w in win:
                    print(f"  bucket {i}: {nb / 2**20:7.2f} MB  released {t:8.3f} ms  window "
                          f"{w:7.3f} ms", file=sys.stderr)
                for n in (2, 4, 8):
                    ex = " ".join(f"{bw} GB/s: {GradSync.exposed_ms(win, n, bw):.3f} ms"
                                  for bw in (100, 300))
                    print(f"  modelled exposed all-reduce time at N={n} (bus bandwidth) {ex}",
                          file=sys.stderr)
        out = {
            "metric": METRIC, "value": cps, "unit": "chars/sec", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": a.dtype if device.type == "cuda" else "fp32",
            "backend": model.backend_name,
            "data": "synthetic (Shakespeare-unigram token stream, random-init weights)",
            "config": {"model": f"{a.layers}-layer {a.model.upper()}-{a.hidden} (vocab {a.vocab})",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": T,
                       "parallelism": f"dp{world}" + ("-zero1" if sharded else "")},
            "vs_torch_nn_lstm_miopen": (cps / (MIOPEN_1GPU_CPS * world)
                                        if (a.model, a.hidden, a.layers, T, B, a.dtype) ==
                                        ("lstm", 512, 2, 128, 256, "bf16") else None),
            "keep_prob": [a.input_keep_prob, a.output_keep_prob],
            "graph": graphed is not None,
            "final_loss": final_loss,
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()
    if a.force_sync and world == 1 and dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
