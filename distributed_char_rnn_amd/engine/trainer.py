"""Training orchestration (reference: ``train(args)``, train.py:73-218).

Per epoch ``e``: ``lr = learning_rate * decay_rate**e``; reset the batch pointer and the TBPTT
state to zeros; per batch feed the previous batch's final state (stateful truncated BPTT,
train.py:185-199), all-reduce gradients (sync DP), clip by global norm + Adam, print the
reference progress line, and save ``model.ckpt-<e*nb+b>`` when ``(e*nb+b) % save_every == 0`` or
on the final batch (train.py:209-217; A-18 kept so ``model.ckpt-14`` exists after 15 one-batch
epochs).

Distributed: sync data parallel over RCCL (see parallel/).  Every rank runs the same number of
steps per epoch (min over ranks); only rank 0 writes config/vocab/checkpoints/logs (fixes the
benign write race of train.py:109-115).  Without ``--tensor_file`` the corpus is sharded
in-process with ``np.array_split`` (any world size).

The loss of step k is read back to the host only after step k+1 has been queued, so the GPU
never idles on the progress print.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import Optional

import numpy as np
import torch

from ..models.char_rnn import CharRNN
from ..models.params import ModelConfig
from ..parallel import process_group, topology
from ..parallel.grad_sync import GradSync
from ..utils import checkpoint as ckpt
from ..utils import data as data_mod
from ..utils import safe_pickle
from ..utils.metrics import MetricsLogger, PhaseProfiler, progress_line
from .graph_step import GraphedStep
from .optim import TFAdam, lr_for_epoch

NEED_BE_SAME = ["model", "rnn_size", "num_layers", "seq_length"]


def _log(msg: str, rank: int = 0):
    if rank == 0:
        print(msg, flush=True)


def make_loader(args, ctx) -> data_mod.TextLoader:
    rank, world = max(ctx.rank, 0), ctx.world_size
    B, T = args.batch_size, args.seq_length
    if args.synthetic_text:
        toks = data_mod.synthetic_tokens(args.synthetic_text, 65, seed=1234)
        if world > 1:
            toks = data_mod.shard(toks, world)[rank]
        return data_mod.ArrayLoader(toks, data_mod.synthetic_chars(65), B, T)
    if args.tensor_file:
        return data_mod.TextLoader(args.data_dir, B, T, tensor_file=args.tensor_file,
                                   verbose=rank == 0)
    if world == 1:
        return data_mod.TextLoader(args.data_dir, B, T)
    # rank 0 preprocesses (may write vocab.pkl / data.npy), the others read after a barrier
    full = None
    if rank == 0:
        full = data_mod.TextLoader(args.data_dir, 1, 1, verbose=True)
    ctx.barrier()
    if full is None:
        full = data_mod.TextLoader(args.data_dir, 1, 1, verbose=False)
    part = data_mod.shard(full.tensor, world)[rank]
    return data_mod.ArrayLoader(part, full.chars, B, T)


def check_init_from(args, loader) -> str:
    """train.py:87-107: required files and model/vocab compatibility."""
    d = args.init_from
    assert os.path.isdir(d), f" {d} must be a a path"
    assert os.path.isfile(os.path.join(d, "config.pkl")), f"config.pkl file does not exist in path {d}"
    assert os.path.isfile(os.path.join(d, "chars_vocab.pkl")), \
        f"chars_vocab.pkl.pkl file does not exist in path {d}"
    prefix = ckpt.latest_checkpoint(d)
    assert prefix, "No checkpoint found"
    saved = safe_pickle.load(os.path.join(d, "config.pkl"))
    for k in NEED_BE_SAME:
        assert vars(saved)[k] == vars(args)[k], \
            f"Command line argument and saved model disagree on '{k}' "
    saved_chars, saved_vocab = safe_pickle.load(os.path.join(d, "chars_vocab.pkl"))
    assert tuple(saved_chars) == tuple(loader.chars), "Data and loaded model disagree on character set!"
    assert dict(saved_vocab) == dict(loader.vocab), "Data and loaded model disagree on dictionary mappings!"
    return prefix


def checkpoint_tensors(model: CharRNN, opt: TFAdam, global_step: int, lr: float, epoch: int,
                       batch: int, state=None):
    """Every tensor of a checkpoint.  ``state`` (``--save_state``): the TBPTT carry after
    ``batch``, as [world, B, H] per (layer, component) -- each data-parallel rank carries its own
    rows (see ``gather_state``) -- so ``--resume_exact`` continues bit-for-bit."""
    t = {}
    t.update(model.store.state_dict())
    t.update(opt.slot_state())
    t["global_step"] = np.array(global_step, dtype=np.int64)
    t["Variable"] = np.array(lr, dtype=np.float32)
    t["dcr/epoch"] = np.array(epoch, dtype=np.int64)
    t["dcr/batch_pointer"] = np.array(batch, dtype=np.int64)
    # the dropout mask counter: --resume_exact continues the mask sequence (same on every rank)
    t["dcr/drop_step"] = np.array(model.drop_step, dtype=np.int64)
    if state is not None:
        for li, st in enumerate(state):
            for si, s in enumerate(st):
                t[f"dcr/state/{li}/{si}"] = s.detach().float().cpu()
    return t


def gather_state(ctx, state):
    """[world, B, H] copies of every state tensor (all ranks' carries), on every rank."""
    out = []
    for st in state:
        comps = []
        for s in st:
            s = s.detach().float().contiguous()
            if ctx.enabled:
                parts = [torch.empty_like(s) for _ in range(ctx.world_size)]
                torch.distributed.all_gather(parts, s)
                full = torch.stack(parts)
            else:
                full = s.unsqueeze(0)
            comps.append(full)
        out.append(tuple(comps))
    return out


def restore_state(model: CharRNN, sd, rank: int, batch: int):
    """The TBPTT carry saved with the checkpoint (``--save_state``), this rank's rows; None if
    the checkpoint has none or it does not match the batch shape."""
    ref = model.zero_state(batch)
    out = []
    for li, st in enumerate(ref):
        comps = []
        for si, z in enumerate(st):
            v = sd.get(f"dcr/state/{li}/{si}")
            if v is None:
                return None
            v = torch.as_tensor(np.asarray(v))
            if v.dim() == z.dim() + 1:  # [world, B, H]
                if rank >= v.shape[0]:
                    return None
                v = v[rank]
            if tuple(v.shape) != tuple(z.shape):
                return None
            comps.append(v.to(device=z.device, dtype=z.dtype))
        out.append(tuple(comps))
    return out


def restore(model: CharRNN, opt: TFAdam, prefix: str):
    sd = ckpt.Saver.restore(prefix)
    model.store.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()
                                 if k in model.store.by_name})
    opt.load_slot_state({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    model.params_changed()
    return sd


def build_model(args, vocab_size: int, device, rank: int = 0) -> CharRNN:
    cfg = ModelConfig(model=args.model, vocab_size=vocab_size, rnn_size=args.rnn_size,
                      num_layers=args.num_layers, input_keep_prob=args.input_keep_prob,
                      output_keep_prob=args.output_keep_prob,
                      clip_norm=getattr(args, "clip_norm", "tf"))
    return CharRNN(cfg, device=device, seed=args.seed, dtype=getattr(args, "dtype", "auto"),
                   rank=rank)


def train(args: argparse.Namespace) -> int:
    topo = topology.from_args(args)
    if topo.role == "ps":
        return process_group.run_ps(topo)
    device = process_group.pick_device(topo, getattr(args, "device", "auto"))
    ctx = process_group.init(topo, device, getattr(args, "dist_backend", "auto"),
                             getattr(args, "dist_timeout", 600.0))
    rank = max(ctx.rank, 0)
    chief = rank == 0
    try:
        return _train(args, ctx, device, rank, chief)
    finally:
        ctx.shutdown()


def _train(args, ctx, device, rank: int, chief: bool) -> int:
    loader = make_loader(args, ctx)
    args.vocab_size = loader.vocab_size
    prefix: Optional[str] = None
    # Only the chief resolves and reads the checkpoint (save_dir need not be on a shared
    # filesystem); the restored step counters, Adam slots and TBPTT carries are broadcast below
    if chief:
        if args.init_from is not None:
            prefix = check_init_from(args, loader)
        elif ctx.world_size > 1 and ckpt.latest_checkpoint(args.save_dir):
            # MonitoredTrainingSession's chief auto-restores from checkpoint_dir
            # (train.py:157-163)
            prefix = ckpt.latest_checkpoint(args.save_dir)

    if chief:
        os.makedirs(args.save_dir, exist_ok=True)
        safe_pickle.dump(args, os.path.join(args.save_dir, "config.pkl"))
        safe_pickle.dump((tuple(loader.chars), dict(loader.vocab)),
                         os.path.join(args.save_dir, "chars_vocab.pkl"))

    model = build_model(args, loader.vocab_size, device, rank)
    # a persistent-kernel timeout makes the optimizer skip its update on device
    opt = TFAdam(model.store, clip=args.grad_clip, guard=model.error_word())
    model.bind_optimizer(opt)  # fused Adam + weight layouts (csrc/tail.hip)
    global_step = 0
    start_epoch, start_batch = 0, 0
    sd = None
    if prefix is not None:
        sd = restore(model, opt, prefix)
        global_step = int(sd.get("global_step", 0))
        if getattr(args, "resume_exact", False):
            start_epoch = int(sd.get("dcr/epoch", 0))
            start_batch = int(sd.get("dcr/batch_pointer", -1)) + 1
            model.drop_step = int(sd.get("dcr/drop_step", 0))
        _log(f"restored {prefix} (global_step {global_step})", rank)

    sharded = getattr(args, "dp_mode", "replicated") == "sharded" and ctx.world_size > 1
    # every rank's error word is MAX-reduced before the optimizer reads it (GradSync.finish /
    # ShardedStep.step): one rank's timed-out recurrence makes every rank skip the update
    sync = GradSync(model.store, ctx.world_size, getattr(args, "bucket_mb", 8.0),
                    getattr(args, "allreduce_dtype", "fp32"),
                    enabled=(ctx.world_size > 1 and not sharded), guard=model.error_word())
    if sync.enabled and sync.guard_view is not None:
        opt.guard = sync.guard_view  # the error words of every rank, summed with the last bucket
    zstep = None
    saved_state = None
    if ctx.world_size > 1:
        # rank 0's restore -> every rank: parameters, Adam slots, step counters (a rank that
        # kept opt.t = 0 would use a different lr_t and diverge; one that kept the batch
        # pointer 0 would run a different number of steps and hang the last all-reduce)
        ctx.broadcast_(model.store.flat)
        ctx.broadcast_(opt.m)
        ctx.broadcast_(opt.v)
        meta = torch.tensor([global_step, opt.t, start_epoch, start_batch, model.drop_step],
                            dtype=torch.int64, device=device if ctx.backend == "nccl" else "cpu")
        ctx.broadcast_(meta)
        global_step, opt.t, start_epoch, start_batch, model.drop_step = (int(v) for v in
                                                                         meta.tolist())
        model.params_changed()
        if start_batch > 0:
            saved_state = _broadcast_state(ctx, model, sd, args.batch_size, device)
    elif sd is not None and start_batch > 0:
        saved_state = restore_state(model, sd, 0, args.batch_size)
    if start_batch > 0 and saved_state is None:
        _log("warning: the checkpoint holds no TBPTT state for this batch shape (train with "
             "--save_state): the resumed epoch continues from a zero state", rank)
    ctx.start_heartbeat(getattr(args, "heartbeat", 0.0))

    nb = ctx.min_int(loader.num_batches)
    if nb != loader.num_batches:
        _log(f"equalising steps per epoch across ranks: {loader.num_batches} -> {nb}", rank)
    total = args.num_epochs * nb
    saver = ckpt.Saver(max_to_keep=5)
    logger = MetricsLogger(args.log_dir, enabled=chief, jsonl_path=getattr(args, "metrics_file", None))
    prof = PhaseProfiler(getattr(args, "profile", False), device)
    chars_per_step = args.batch_size * args.seq_length * ctx.world_size
    log_every = max(1, getattr(args, "log_every", 1))
    summary_every = getattr(args, "summary_every", 100)
    max_steps = getattr(args, "max_steps", 0)
    steps_done = 0
    # Only logged steps (every --log_every, the last, and checkpoint steps) read their loss back:
    # a logged step is flushed after the NEXT step was enqueued, so the host never drains the
    # GPU, and time/batch is the mean over the steps since the previous logged step.
    pending = None  # (global_step, epoch, loss_tensor, steps in its span, span start)
    span_t0, span_n = None, 0

    def flush(p, now):
        gs, e, loss_t, n, ts = p
        dt = (now - ts) / max(n, 1)
        loss = float(loss_t)
        if chief and (gs % log_every == 0 or gs == total):
            print(progress_line(gs, total, e, loss, dt, chars_per_step / max(dt, 1e-9)), flush=True)
        logger.log({"step": gs, "epoch": e, "loss": loss, "time_per_batch": dt,
                    "chars_per_sec": chars_per_step / max(dt, 1e-9), "rank_world": ctx.world_size})
        logger.scalar("train_loss", loss, gs)

    if sharded:
        from ..parallel.zero import ShardedStep

        zstep = ShardedStep(model.store, opt, ctx.world_size, rank,
                            wire=getattr(args, "allreduce_dtype", "fp32"),
                            bucket_mb=getattr(args, "bucket_mb", 8.0), guard=model.error_word())
        _log(f"sharded optimizer: shard {zstep.shard} of {model.store.numel} elements in "
             f"{len(zstep.buckets)} buckets", rank)
    # data parallelism: poll the persistent kernels' error word after the exchange has folded
    # every rank's word into each rank's own, so all ranks raise on the same step
    defer_poll = ctx.world_size > 1 and hasattr(model.backend, "defer_err_poll")
    if defer_poll:
        model.backend.defer_err_poll = True
    # --graph: the whole step (fwd, head, BPTT, weight grads, clip + Adam) as one replayed
    # hipGraph; summary steps that want the logits run eagerly
    graphed = None
    gmode = getattr(args, "graph", "off")
    if gmode == "auto" and args.batch_size * args.seq_length * args.rnn_size > GRAPH_AUTO_MAX_WORK:
        # a step this large is not launch-bound: the replay's input / state / loss copies cost
        # more than the launches they save (headline shape, same box: eager 1.394-1.412 vs
        # graph 1.454-1.456 ms per train.py step; bench.py 1.390-1.396 vs --graph 1.425-1.436)
        gmode = "off"
    if gmode != "off":
        ok, why = GraphedStep.supported(model, ctx.world_size)
        if ok:
            graphed = GraphedStep(model, opt, log=lambda m: _log(m, rank))
        elif args.graph == "on":
            _log(f"--graph on: not available ({why}); eager steps", rank)
    dev_batches = _device_batches(loader, nb, device)
    stop = False
    state = None
    for e in range(start_epoch, args.num_epochs):
        lr = lr_for_epoch(args.learning_rate, args.decay_rate, e)
        loader.reset_batch_pointer()
        state = model.zero_state(args.batch_size)
        b0 = start_batch if e == start_epoch else 0
        if b0:
            loader.pointer = b0
            if saved_state is not None:  # the carry of the interrupted run's batch b0 - 1
                state = saved_state
        for b in range(b0, nb):
            t0 = time.time()
            if span_t0 is None:
                span_t0 = t0
            x, y = loader.next_batch()
            if dev_batches is not None:  # the same batch, already resident on the device
                x, y = dev_batches[0][b], dev_batches[1][b]
            want = chief and summary_every > 0 and (global_step % summary_every == 0)
            if zstep is not None:  # sharded optimizer step (ZeRO-1): the backward launches
                # each bucket's reduce-scatter as soon as its gradients are final
                with prof.phase("fwd_bwd"):
                    loss_t, state, extras = _step(model, x, y, state, zstep, want)
                with prof.phase("sharded_step"):
                    zstep.step(lr)
            elif graphed is not None and not want:
                with prof.phase("graph_step"):
                    loss_t, state = graphed(x, y, state, lr)
                extras = None
            else:
                with prof.phase("fwd_bwd"):
                    loss_t, state, extras = _step(model, x, y, state, sync, want)
                with prof.phase("grad_sync"):
                    gs = sync.finish(defer_scale=True)
                with prof.phase("optimizer"):
                    opt.step(lr, grad_scale=gs)
            if defer_poll:
                model.poll_errors()
            global_step += 1
            steps_done += 1
            process_group.maybe_inject_fault(rank, global_step)
            if pending is not None:
                flush(pending, t0)
                pending = None
            span_n += 1
            if want and extras:
                if extras.get("logits") is not None:
                    logger.histogram("logits", extras["logits"].float().cpu().numpy(), global_step)
                if extras.get("loss") is not None:
                    logger.histogram("loss", extras["loss"].float().cpu().numpy(), global_step)
            step_idx = e * nb + b
            last = (e == args.num_epochs - 1 and b == nb - 1)
            if max_steps and steps_done >= max_steps:
                last, stop = True, True
            saving = step_idx % args.save_every == 0 or last
            if global_step % log_every == 0 or global_step == total or saving:
                pending = (global_step, e, loss_t, span_n, span_t0)
                span_t0, span_n = None, 0
            if saving:
                if pending is not None:
                    flush(pending, time.time())
                    pending = None
                model.check_errors()  # never checkpoint weights of a timed-out step
                save_st = None
                if zstep is not None:
                    zstep.gather_slots()  # collective: the chief saves the full Adam slots
                if getattr(args, "save_state", False):
                    save_st = gather_state(ctx, state)  # collective: every rank
                if chief:
                    tensors = checkpoint_tensors(model, opt, global_step, lr, e, b, save_st)
                    path = saver.save(args.save_dir, tensors, step_idx)
                    print("model saved to {}".format(os.path.join(args.save_dir, "model.ckpt")),
                          flush=True)
                    logger.log({"step": global_step, "saved": path})
            if stop:
                break
        if stop:
            break
    if pending is not None:
        flush(pending, time.time())
    model.check_errors()
    if prof.enabled and chief:
        print(prof.table(), flush=True)
    logger.close()
    return 0


DEVICE_BATCHES_MAX_BYTES = 4 << 30
# --graph auto replays captured steps only below this B·T·H (launch-bound shapes, e.g. the
# reference default B = 50, T = 50, H = 128)
GRAPH_AUTO_MAX_WORK = 1 << 21


def _device_batches(loader, nb: int, device: torch.device):
    """The epoch's x / y batches as two device-resident int32 [nb, B, T] tensors, uploaded
    once (the reference's feed_dict copies every batch, train.py:203; here a step then needs no
    pinning or host-to-device copy).  None on the CPU, or when the batches would take more than
    DEVICE_BATCHES_MAX_BYTES of HBM (per-step copies then, models/char_rnn.py _as_ids)."""
    if device.type != "cuda" or nb == 0:
        return None
    nbytes = 2 * 4 * nb * int(np.asarray(loader.x_batches[0]).size)
    if nbytes > DEVICE_BATCHES_MAX_BYTES:
        return None
    up = lambda bs: torch.from_numpy(  # noqa: E731
        np.ascontiguousarray(np.stack(bs[:nb]), dtype=np.int32)).to(device)
    return up(loader.x_batches), up(loader.y_batches)


def _broadcast_state(ctx, model: CharRNN, sd, batch: int, device):
    """Rank 0 holds the checkpoint's [world, B, H] carries: broadcast them, each rank keeps its
    own rows.  None (on every rank) when the checkpoint has none."""
    ref = model.zero_state(batch)
    have = torch.zeros(1, dtype=torch.int64, device=device if ctx.backend == "nccl" else "cpu")
    full = None
    if ctx.rank == 0 and sd is not None:
        full = restore_state(model, sd, 0, batch)  # shape check on rank 0's rows
        if full is not None and all(np.asarray(sd[f"dcr/state/{li}/{si}"]).ndim == 3 and
                                    np.asarray(sd[f"dcr/state/{li}/{si}"]).shape[0] == ctx.world_size
                                    for li, st in enumerate(ref) for si in range(len(st))):
            have.fill_(1)
    ctx.broadcast_(have)
    if not int(have.item()):
        return None
    out = []
    for li, st in enumerate(ref):
        comps = []
        for si, z in enumerate(st):
            buf = torch.empty((ctx.world_size,) + tuple(z.shape), dtype=torch.float32,
                              device=z.device if ctx.backend == "nccl" else "cpu")
            if ctx.rank == 0:
                buf.copy_(torch.as_tensor(np.asarray(sd[f"dcr/state/{li}/{si}"])))
            ctx.broadcast_(buf)
            comps.append(buf[ctx.rank].to(device=z.device, dtype=z.dtype).clone())
        out.append(tuple(comps))
    return out


def _step(model: CharRNN, x, y, state, sync, want_extras: bool):
    """``sync``: a GradSync (replicated) or ShardedStep (sharded): both are reset here and
    driven by the backward's readiness callbacks."""
    sync.reset()
    loss, new_state, extras = model.train_step(x, y, state, sync, want_extras=want_extras)
    return loss, new_state, (extras if want_extras else None)


def main(argv=None) -> int:
    from ..utils.config import train_parser

    args = train_parser().parse_args(argv)
    return train(args)


if __name__ == "__main__":
    sys.exit(main())
