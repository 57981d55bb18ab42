"""One process per GPU without an external launcher (torchrun-style), shared by bench.py and
train.py.

The reference gets its per-GPU processes from Lightning: `trainer.devices > 1` turns on DDP
(/root/reference/train.py:630-639) and Lightning re-launches the script once per device. Here
`launch_ranks` does the same before the parent touches the GPU: it starts N children of the same
script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, rank r binds cuda:r,
and the parent only waits (its exit code is the first failing rank's). Never exec'ing from a
process that initialised HIP is the point: the children are fresh interpreters.
"""
import os
import signal
import socket
import subprocess
import sys
import time


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, script, argv, extra_env=None):
    """Start `n` rank processes of `script argv...`, wait for all, return the exit status (first
    failing rank's; the others are sent SIGTERM, as a rank stuck in a collective would hang)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script)] + list(argv),
                                      env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc if rc >= 0 else 128 - rc


def dist_backend():
    """"nccl" (RCCL over xGMI) unless DNA_DIST_BACKEND names another (gloo: the rehearsal that
    runs every rank on the visible GPUs round-robin, e.g. two ranks on a one-GPU box)."""
    return os.environ.get("DNA_DIST_BACKEND", "nccl")


def rank_device_index(local_rank):
    """GPU of this rank: cuda:local_rank, or round-robin over the visible GPUs for a non-RCCL
    rehearsal (device_count() does not initialise HIP on this image)."""
    if dist_backend() == "nccl":
        return local_rank
    import torch
    return local_rank % max(1, torch.cuda.device_count())


def wants_process_group(world):
    """A process group exists for world > 1, and at world 1 when DNA_DDP_FORCE=1 asks the
    gradient reducer to run its collectives anyway (the one-GPU RCCL rehearsal)."""
    return world > 1 or os.environ.get("DNA_DDP_FORCE", "0") == "1"


def init_rank_process_group(local_rank):
    """Bind this rank's GPU and join the process group (RCCL binds the device at init)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:  # a forced world-1 group started without a launcher
        os.environ["MASTER_PORT"] = str(free_port())
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    hang = os.environ.get("DNA_HANG_DUMP")
    if hang:  # diagnostics: every thread's Python stack on stderr if the rank is still alive then
        import faulthandler
        faulthandler.dump_traceback_later(int(hang), repeat=True)
    dev = rank_device_index(local_rank)
    torch.cuda.set_device(dev)
    if dist_backend() == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(dist_backend())
    return torch.device("cuda", dev)


def flat_digest(flat):
    """sha256 of a flat parameter buffer's bytes + its float64 sum (debug dumps that show two
    ranks hold identical parameters)."""
    import hashlib
    import torch
    t = flat.detach().contiguous().cpu().view(-1)
    return {"sha256": hashlib.sha256(t.view(torch.uint8).numpy().tobytes()).hexdigest(),
            "sum": float(t.double().sum()), "numel": int(t.numel())}
