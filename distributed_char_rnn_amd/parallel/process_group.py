"""Process-group lifecycle: rendezvous, RCCL/gloo backend, heartbeats, ps role, teardown.

Replaces the reference's TF gRPC cluster (``tf.train.ClusterSpec`` + ``tf.train.Server``,
train.py:117-135) and the chief/non-chief session logic of ``MonitoredTrainingSession``
(train.py:157-163).  One process drives one GPU; collectives go through ``torch.distributed``
with the ``nccl`` backend, which is RCCL over xGMI on ROCm, or ``gloo`` for CPU tests.

Failure detection (the reference has none -- a dead PS or worker leaves the
others blocked in gRPC, train.py:129-130): every collective carries ``--dist_timeout``; with
``--heartbeat S`` each rank refreshes ``hb/<rank>`` in the store every S seconds, rank 0 marks
a rank whose heartbeat is older than 3·S as lost by setting ``abort`` in the store, and every
rank's heartbeat thread that sees ``abort`` (or loses the store, i.e. rank 0 died) ends its
process with ``EXIT_PEER_LOST`` instead of waiting out the collective timeout.  Recovery is
checkpoint based: relaunch all ranks with ``--init_from <save_dir>`` (``--resume_exact``
continues at the saved epoch/batch).  ``DCR_FAULT=<rank>:<step>`` kills that rank at that global
step (fault injection for the tests).
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist

from .topology import Topology


EXIT_PEER_LOST = 75  # EX_TEMPFAIL: a peer died; relaunch every rank with --init_from


def maybe_inject_fault(rank: int, global_step: int, log=print):
    """``DCR_FAULT=<rank>:<step>``: simulate a crash of ``rank`` at ``global_step``."""
    spec = os.environ.get("DCR_FAULT", "")
    if not spec:
        return
    r, _, st = spec.partition(":")
    if int(r) == rank and int(st) == global_step:
        log(f"[fault] injected crash of rank {rank} at step {global_step}")
        os._exit(17)


class DistContext:
    def __init__(self, topo: Topology, device: torch.device, backend: str,
                 store: Optional[dist.Store] = None):
        self.topo = topo
        self.device = device
        self.backend = backend
        self.store = store
        self._hb_stop = threading.Event()
        self._hb_thread: Optional[threading.Thread] = None

    @property
    def rank(self) -> int:
        return self.topo.rank

    @property
    def world_size(self) -> int:
        return self.topo.world_size

    @property
    def enabled(self) -> bool:
        return dist.is_available() and dist.is_initialized() and self.world_size > 1

    def barrier(self):
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_scalar(self, v: float, op=dist.ReduceOp.SUM) -> float:
        if not self.enabled:
            return v
        t = torch.tensor([v], dtype=torch.float64 if self.backend == "gloo" else torch.float32,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=op)
        return float(t.item())

    def min_int(self, v: int) -> int:
        if not self.enabled:
            return v
        t = torch.tensor([v], dtype=torch.int64,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if self.enabled:
            dist.broadcast(t, src)
        return t

    # -- heartbeats ------------------------------------------------------------------------
    def start_heartbeat(self, period: float, log=print):
        if period <= 0 or self.store is None or not self.enabled:
            return

        def lost(msg):
            log(f"[heartbeat] rank {self.rank}: {msg}; exiting with {EXIT_PEER_LOST} "
                "(relaunch all ranks with --init_from)")
            os._exit(EXIT_PEER_LOST)

        def run():
            # Each rank publishes a monotonically increasing beat counter; rank 0 notes, on its
            # own monotonic clock, when each rank's counter last moved (no cross-host wall
            # clocks: skew between hosts cannot declare a healthy rank dead)
            failures, beat = 0, 0
            last_seen = {}  # rank -> (counter, monotonic time it last changed)
            while not self._hb_stop.wait(period):
                try:
                    beat += 1
                    self.store.set(f"hb/{self.rank}", str(beat))
                    if self.store.check(["abort"]):
                        lost("abort: " + self.store.get("abort").decode())
                    if self.rank == 0:
                        now = time.monotonic()
                        for r in range(self.world_size):
                            try:
                                c = int(self.store.get(f"hb/{r}").decode())
                            except Exception:
                                continue
                            prev = last_seen.get(r)
                            if prev is None or prev[0] != c:
                                last_seen[r] = (c, now)
                            elif now - prev[1] > 3 * period:
                                msg = f"rank {r} silent for {now - prev[1]:.1f}s"
                                self.store.set("abort", msg)
                                lost(msg)
                    failures = 0
                except Exception:
                    if self._hb_stop.is_set():
                        return
                    failures += 1
                    if failures >= 3:  # the store (rank 0 / ps) is gone
                        lost("rendezvous store unreachable")

        self.store.set(f"hb/{self.rank}", "0")
        self._hb_thread = threading.Thread(target=run, daemon=True, name="dcr-heartbeat")
        self._hb_thread.start()

    def shutdown(self):
        self._hb_stop.set()
        if self.store is not None and self.topo.store_host_is_ps and self.topo.role == "worker":
            try:
                self.store.add("workers_done", 1)
            except Exception:
                pass
        if dist.is_available() and dist.is_initialized():
            try:
                self.barrier()
            except Exception:
                pass
            dist.destroy_process_group()


def pick_device(topo: Topology, requested: str = "auto", log=print) -> torch.device:
    if requested == "cpu":
        return torch.device("cpu")
    if requested in ("auto", "cuda") and torch.cuda.is_available():
        n = torch.cuda.device_count()
        local_world = topo.local_world_size
        if local_world > n:
            # more local ranks than GPUs: ranks share a device.  The persistent recurrent
            # kernels need every CU of the chip (one workgroup per CU, co-resident grids), so two
            # processes' grids on one GPU spin into the timeout: use the per-step kernels.
            # (DCR_GPU_SHARE keeps them: persistent launches serialised across processes by a
            # file lock, engine/native/backend.py SharedGpuOps -- a test mode)
            if (os.environ.get("DCR_RECURRENCE", "auto") in ("auto", "single")
                    and not os.environ.get("DCR_GPU_SHARE")):
                log(f"[rank {topo.rank}] {local_world} local ranks share {n} GPU(s): persistent "
                    "kernels disabled (DCR_RECURRENCE=step); run one rank per GPU for speed")
                os.environ["DCR_RECURRENCE"] = "step"
        dev = torch.device("cuda", topo.local_rank % max(n, 1))
        torch.cuda.set_device(dev)
        return dev
    if requested == "cuda":
        raise RuntimeError("--device cuda requested but no GPU is visible")
    return torch.device("cpu")


def init(topo: Topology, device: torch.device, backend: str = "auto",
         timeout_s: float = 600.0) -> DistContext:
    if backend == "auto":
        backend = "nccl" if device.type == "cuda" else "gloo"
    if not topo.distributed:
        return DistContext(topo, device, backend)
    timeout = datetime.timedelta(seconds=timeout_s)
    if topo.from_env:
        dist.init_process_group(backend=backend, timeout=timeout,
                                device_id=device if device.type == "cuda" else None)
        try:  # torchrun's rendezvous store, for heartbeats
            store = dist.distributed_c10d._get_default_store()
        except Exception:
            store = None
        return DistContext(topo, device, backend, store=store)
    is_master = (topo.rank == 0 and not topo.store_host_is_ps)
    store = dist.TCPStore(topo.master_addr, topo.master_port, world_size=None,
                          is_master=is_master, timeout=timeout, wait_for_workers=False)
    dist.init_process_group(backend=backend, store=store, rank=topo.rank,
                            world_size=topo.world_size, timeout=timeout,
                            device_id=device if device.type == "cuda" else None)
    return DistContext(topo, device, backend, store=store)


def run_ps(topo: Topology, timeout_s: float = 86400.0, log=print) -> int:
    """The ``--job_name ps`` role: host the rendezvous store, return when workers finish."""
    store = dist.TCPStore(topo.master_addr, topo.master_port, world_size=None, is_master=True,
                          timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
    log(f"ps: rendezvous store listening on {topo.master_addr}:{topo.master_port} "
        f"for {topo.world_size} workers")
    t0 = time.time()
    while True:
        try:
            done = store.add("workers_done", 0)
        except Exception:
            done = 0
        if done >= topo.world_size:
            log("ps: all workers finished")
            return 0
        if time.time() - t0 > timeout_s:
            log("ps: timed out waiting for workers")
            return 1
        time.sleep(0.5)


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default
