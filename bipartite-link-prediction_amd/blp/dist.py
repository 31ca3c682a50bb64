"""Multi-GPU plumbing: one process per GPU, launched by torchrun.

Two modes, both with no collective on the scoring data path:

* replicas (configs 2-4): every rank builds the whole graph and scores its own sources;
  torch.distributed (gloo, CPU tensors) is used only for the barrier and the max / sum of
  the timings (weak scaling).
* row-block sharded ingest (config 5): rank r owns the users of block r (contiguous ids,
  balanced by work) and produces only their edges; ONE exchange step -- an RCCL
  all-gather of the per-rank edge partials over xGMI (backend "nccl" is RCCL on ROCm) --
  gives every rank the complete edge list in HBM, from which libblp builds the CSR on the
  device (blp_csr_from_edges_device). After the exchange all scoring is rank-local.

torch is plumbing here (process group, device buffers for the collective); the graph and
every kernel live in libblp.so.
"""
import contextlib
import os
import sys

import numpy as np

from . import synth


@contextlib.contextmanager
def stdout_to_stderr():
    """Point file descriptor 1 at stderr: gloo's connection banner and RCCL's version banner
    (printed when its communicator forms, at the first collective) go to stdout from C++, and
    the bench's stdout is its one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class Dist:
    """Rank / world from the torchrun environment; CPU (gloo) reductions; optional RCCL group."""

    def __init__(self, exchange=False, collective_at_world1=False):
        """exchange: form the RCCL group the config-5 exchange uses (BLP_EXCHANGE_BACKEND=gloo
        rehearses it over gloo instead). collective_at_world1: form the process group even
        for a single rank, so the exchange runs the real collective (RCCL's all-gather over
        one rank) rather than returning the local partial -- the code path of N ranks,
        exercised on a one-GPU box."""
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.exchange = exchange
        self.td = None
        self.cpu_group = None
        if self.world == 1 and exchange and collective_at_world1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if self.world > 1 or (exchange and collective_at_world1):
            import torch.distributed as td

            self.td = td
            # gloo's C++ layer prints its connection banner on stdout; the bench's stdout is
            # its one JSON line, so stdout is pointed at stderr while the groups form
            with stdout_to_stderr():
                if exchange and os.environ.get("BLP_EXCHANGE_BACKEND", "nccl") == "nccl":
                    import torch

                    torch.cuda.set_device(self.local)
                    td.init_process_group("nccl")
                    self.cpu_group = td.new_group(backend="gloo")
                    self.backend = "nccl"
                else:
                    td.init_process_group("gloo")
                    self.backend = "gloo"
                td.barrier(group=self.cpu_group)  # every rank connected before stdout returns
        else:
            self.backend = None

    # --------------------------------------------------------------- CPU reductions
    def barrier(self):
        if self.world > 1:
            self.td.barrier(group=self.cpu_group)

    def _reduce(self, v, op):
        if self.world == 1:
            return v
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64)
        self.td.all_reduce(t, op=op, group=self.cpu_group)
        return float(t.item())

    def max(self, v):
        return self._reduce(v, self.td.ReduceOp.MAX if self.td else None)

    def sum(self, v):
        return self._reduce(v, self.td.ReduceOp.SUM if self.td else None)

    def allgather_int(self, v):
        """[v_0, ..., v_{world-1}] (int64, over the CPU group)."""
        if self.world == 1:
            return [int(v)]
        import torch

        out = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        self.td.all_gather(out, torch.tensor([int(v)], dtype=torch.int64), group=self.cpu_group)
        return [int(t.item()) for t in out]

    def broadcast_bytes(self, b, src=0):
        """Rank src's bytes on every rank (over the CPU group), e.g. libblp's RCCL id."""
        if self.world == 1:
            return b
        box = [b]
        self.td.broadcast_object_list(box, src=src, group=self.cpu_group)
        return box[0]

    def close(self):
        if self.td is not None and self.td.is_initialized():
            self.td.destroy_process_group()


def _free_port():
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def user_blocks(n_users, world, work=None):
    """Contiguous user blocks [b[r], b[r+1]) for `world` ranks, balanced by cumulative
    work (sum_{b in N(u)} d_b + sum over pairs d_v) when given, else by count."""
    if work is None:
        return np.array([n_users * r // world for r in range(world + 1)], np.int64)
    c = np.concatenate([[0], np.cumsum(np.asarray(work, np.float64))])
    targets = c[-1] * np.arange(world + 1) / world
    b = np.searchsorted(c, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, n_users
    return np.maximum.accumulate(b)


def block_review_edges(users, businesses, draws, lo, hi, seed=0, zipf=0.8):
    """The edge partial of user block [lo, hi): the draws of synth.review_edges' distribution
    (uniform user, Zipf business popularity) whose user falls in the block, generated
    block-locally -- round(draws * (hi - lo) / users) draws, users uniform in the block.
    The union over a partition is a graph of the same distribution (not the same sample as
    the single-process generator)."""
    n = int(round(draws * (hi - lo) / float(users)))
    p = synth.popularity(businesses, zipf)
    cdf = np.cumsum(p)
    u = np.empty(n, np.int64)
    b = np.empty(n, np.int64)
    step = 25_000_000

    def chunk(i):  # each chunk its own seeded stream: the result does not depend on the thread count
        s, e = i * step, min(n, (i + 1) * step)
        rng = np.random.default_rng([seed, lo, hi, i])
        u[s:e] = rng.integers(lo, hi, e - s)
        b[s:e] = np.minimum(np.searchsorted(cdf, rng.random(e - s)), businesses - 1) + users

    from concurrent.futures import ThreadPoolExecutor

    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(workers) as ex:  # numpy's bulk draws and searchsorted release the GIL
        list(ex.map(chunk, range((n + step - 1) // step)))
    return u, b


def allgather_edges(dist, a_local, b_local):
    """The exchange step: all-gather every rank's edge partial (int32 endpoints).

    nccl (RCCL over xGMI): device tensors in, device tensors out (torch.int32 on the local
    GPU) -- the caller hands their pointers to blp_csr_from_edges_device. gloo: CPU tensors.
    Partials are padded to the largest count for all_gather_into_tensor (RCCL has no
    all-gather-v); the counts go first over the CPU group. Returns (a, b, counts)."""
    import torch

    counts = dist.allgather_int(len(a_local))
    mx = max(counts) if counts else 0
    on_gpu = dist.backend == "nccl" or (dist.world == 1 and dist.exchange and torch.cuda.is_available())
    dev = torch.device("cuda", dist.local) if on_gpu else torch.device("cpu")
    mine = torch.full((2, max(mx, 1)), -1, dtype=torch.int32, device=dev)
    if len(a_local):
        mine[0, : len(a_local)] = torch.as_tensor(np.asarray(a_local, np.int32)).to(dev)
        mine[1, : len(b_local)] = torch.as_tensor(np.asarray(b_local, np.int32)).to(dev)
    if dist.td is None:  # a single rank without a process group: nothing to exchange
        return mine[0, : counts[0]].contiguous(), mine[1, : counts[0]].contiguous(), counts
    out = torch.empty((dist.world, 2, max(mx, 1)), dtype=torch.int32, device=dev)
    if dist.backend == "nccl":
        with stdout_to_stderr():  # the communicator forms here (RCCL's banner)
            dist.td.all_gather_into_tensor(out, mine)
            torch.cuda.synchronize(dev)
    else:
        dist.td.all_gather(list(out.unbind(0)), mine, group=dist.cpu_group)
    a = torch.cat([out[r, 0, : counts[r]] for r in range(dist.world)])
    b = torch.cat([out[r, 1, : counts[r]] for r in range(dist.world)])
    return a, b, counts
