"""`bench.py --gpus N` as its own launcher: one process per GPU without torchrun.

The driver runs `python3 bench.py --gpus N ...` for single-node benches and
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...` for the scaling
runs. Both must give N ranks. Under a launcher (WORLD_SIZE in the environment) the process is
one rank and `--gpus` must equal WORLD_SIZE. Without one and with N > 1, the parent starts N
fresh `python bench.py` children (subprocess: fork + exec of a new interpreter, from a
parent that has made no HIP call, so no process that touched the GPU is ever replaced),
each with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set
as torchrun sets them, and waits. Rank 0 inherits the parent's stdout and prints the one
result line; the parent prints nothing on stdout. When a child fails, the others (likely
blocked in a collective) get SIGTERM after a grace period, then SIGKILL; the parent exits
with the first failing child's status. The reference's only parallelism is the chunked
query split of `static-search-tree/src/bin/bench.rs:558-573` (rayon threads); ranks here
play that role one GPU each.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


class WorldMismatch(SystemExit):
    pass


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def resolve_world(gpus, environ=None):
    """(world_size, rank, local_rank) of this process, checked against --gpus.

    WORLD_SIZE unset: (gpus or 1, 0, 0), and the caller spawns when that is > 1.
    WORLD_SIZE set (torchrun, or our own children): --gpus, when given, must equal it."""
    env = os.environ if environ is None else environ
    if "WORLD_SIZE" not in env:
        return (gpus or 1), 0, 0
    ws = int(env["WORLD_SIZE"])
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    if gpus is not None and gpus != ws:
        raise WorldMismatch(f"bench: --gpus {gpus} but the launcher's WORLD_SIZE is {ws}; "
                            f"run `python bench.py --gpus N` alone or pass the same N to both")
    if not (0 <= rank < ws and 0 <= local < ws):
        raise WorldMismatch(f"bench: RANK {rank} / LOCAL_RANK {local} outside WORLD_SIZE {ws}")
    return ws, rank, local


def needs_spawn(gpus, environ=None) -> bool:
    env = os.environ if environ is None else environ
    return "WORLD_SIZE" not in env and (gpus or 1) > 1


def _exit_status(rc: int) -> int:
    return rc if rc > 0 else (128 + (-rc) if rc < 0 else 0)


def spawn_ranks(n: int, script: str, argv, grace_s: float | None = None, python: str | None = None) -> int:
    """Run `python script argv...` as N ranks on this node; return the job's exit status
    (0 iff every rank exited 0)."""
    if grace_s is None:
        grace_s = float(os.environ.get("SAS_LAUNCH_GRACE_S", "20"))
    port = free_port()
    procs = []
    base = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([python or sys.executable, script, *argv], env=env))

    def stop(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    # a signal to the parent (a driver timeout) reaches every rank
    old = {s: signal.getsignal(s) for s in (signal.SIGTERM, signal.SIGINT)}

    def forward(sig, _frame):
        stop(sig)
        raise SystemExit(128 + sig)
    for s in old:
        signal.signal(s, forward)
    status = 0
    try:
        failed_at = None
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                break
            bad = [c for c in codes if c not in (None, 0)]
            if bad and failed_at is None:
                failed_at = time.monotonic()
                status = _exit_status(bad[0])
                print(f"[launch] a rank exited {bad[0]}; stopping the others in {grace_s:.0f} s",
                      file=sys.stderr, flush=True)
            if failed_at is not None:
                waited = time.monotonic() - failed_at
                if waited > grace_s + 10:
                    stop(signal.SIGKILL)
                elif waited > grace_s:
                    stop(signal.SIGTERM)
            time.sleep(0.05)
        for r, p in enumerate(procs):
            if p.returncode != 0:
                print(f"[launch] rank {r} exit {p.returncode}", file=sys.stderr, flush=True)
                if status == 0:
                    status = _exit_status(p.returncode)
    finally:
        # normal exit: every rank is done already; after a forwarded signal give them 5 s
        deadline = time.monotonic() + 5
        for p in procs:
            try:
                p.wait(timeout=max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                pass
        stop(signal.SIGKILL)
        for p in procs:
            p.wait()
        for s, h in old.items():
            signal.signal(s, h)
    return status


def probe_main(args, emit, log) -> int:
    """`bench.py --workload launch_probe`: the launcher's CPU rehearsal. Every rank joins a
    gloo group, runs a stub step through bench's own timed_loop (barrier + MAX all-reduce),
    and rank 0 prints one line with what each rank saw. `--probe-fail-rank R` makes rank R
    exit 3 before joining (the others then block in the rendezvous until the launcher stops
    them)."""
    import torch
    import torch.distributed as dist
    from benchlib.common import timed_loop
    ws, rank, local = resolve_world(args.gpus)
    if args.probe_fail_rank == rank:
        log(f"rank {rank}: failing on purpose (--probe-fail-rank)")
        return 3
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        def step():
            time.sleep(0.002 * (1 + rank))

        def reduce_max(x):
            t = torch.tensor([x], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        el = timed_loop(step, args.steps, args.warmup, lambda: None, dist.barrier, reduce_max)
        mine = {"rank": rank, "local_rank": local, "env_world_size": int(os.environ.get("WORLD_SIZE", "1")),
                "group_world_size": dist.get_world_size(), "pid": os.getpid(), "elapsed_s": el}
        seen = [None] * ws
        dist.all_gather_object(seen, mine)
        if rank == 0:
            emit({"metric": "launch_probe", "n_gpus": dist.get_world_size(), "steps": args.steps,
                  "warmup": args.warmup, "elapsed_s": el, "ranks": seen})
        dist.barrier()
    finally:
        dist.destroy_process_group()
    return 0
