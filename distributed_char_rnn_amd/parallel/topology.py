"""Map the reference's parameter-server flags (and torchrun env vars) onto a synchronous
data-parallel world of one process per GPU.

Reference (train.py:117-135): ``--distributed --ps_hosts H:P --worker_hosts H:P,H:P,...
--job_name {ps,worker} --task_index i`` builds a TF gRPC cluster with async PS updates.  Here:

* ``worker i``  -> rank ``i`` of ``world = len(worker_hosts)``; device ``cuda:(i % gpus)``;
* ``ps 0``      -> hosts the rendezvous key-value store at ``ps_hosts[0]`` and exits once every
                   worker has finished (fixes the ``server.join()`` hang, A-16);
* without a ps, worker 0 hosts the store at ``worker_hosts[0]``;
* under ``torchrun`` (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT in the environment)
  the environment wins and the PS flags are ignored.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional


@dataclass
class Topology:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    role: str = "worker"  # worker | ps
    store_host_is_ps: bool = False
    from_env: bool = False
    local_world_size: int = 1  # ranks on this host (more than its GPUs => shared devices)

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.role == "ps"

    @property
    def is_chief(self) -> bool:
        return self.rank == 0 and self.role == "worker"


def _split_hostport(s: str):
    s = s.strip()
    if ":" not in s:
        return s, 29500
    h, p = s.rsplit(":", 1)
    return h, int(p)


def from_env() -> Optional[Topology]:
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return Topology(rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]),
                        local_rank=int(os.environ.get("LOCAL_RANK", os.environ["RANK"])),
                        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                        master_port=int(os.environ.get("MASTER_PORT", 29500)), from_env=True,
                        local_world_size=int(os.environ.get("LOCAL_WORLD_SIZE",
                                                            os.environ["WORLD_SIZE"])))
    return None


def from_args(args) -> Topology:
    env = from_env()
    if env is not None:
        return env
    if not getattr(args, "distributed", False):
        return Topology()
    if not args.worker_hosts:
        raise ValueError("--distributed requires --worker_hosts")
    workers = [w for w in args.worker_hosts.split(",") if w.strip()]
    if args.job_name not in ("ps", "worker"):
        raise ValueError("--distributed requires --job_name ps|worker")
    if args.task_index is None:
        raise ValueError("--distributed requires --task_index")
    if args.ps_hosts:
        host, port = _split_hostport(args.ps_hosts.split(",")[0])
        ps = True
    else:
        host, port = _split_hostport(workers[0])
        ps = False
    if args.job_name == "ps":
        return Topology(rank=-1, world_size=len(workers), local_rank=0, master_addr=host,
                        master_port=port, role="ps", store_host_is_ps=True)
    if not 0 <= args.task_index < len(workers):
        raise ValueError(f"task_index {args.task_index} out of range for {len(workers)} workers")
    hosts = [_split_hostport(w)[0] for w in workers]
    mine = hosts[args.task_index]
    local = [i for i, h in enumerate(hosts) if h == mine]
    return Topology(rank=args.task_index, world_size=len(workers),
                    local_rank=local.index(args.task_index), master_addr=host, master_port=port,
                    role="worker", store_host_is_ps=ps, local_world_size=len(local))
