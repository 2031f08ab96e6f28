"""Compaction-job sharding across GPUs (SURVEY.md §8e, configs[4]).

SSTs are independent: L0 flush emits one per memtable and compaction a sequence of output SSTs
(flush.rs:68-146, compactor_executor.rs:787-871), and the bloom filter is per SST
(sst_builder.rs:390-403).  So a job of J SSTs shards over N ranks with no collective on the data
path: SST j goes to rank j mod N, every rank encodes its own share, and the whole-job rate is
Σ logical bytes of all ranks ÷ the slowest rank's wall time.  The only collectives are the timing
barrier and a max / sum of scalars (RCCL on the GPU box, gloo in the CPU tests).
"""


def assign(num_ssts, world):
    """SST ids per rank: SST j -> rank j mod world (configs[4]: 64 SSTs, 8 per GPU at world 8)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    return [list(range(r, num_ssts, world)) for r in range(world)]


def share(num_ssts, world, rank):
    return assign(num_ssts, world)[rank]


def aggregate(dist, logical_bytes, elapsed_s, device=None):
    """(total logical bytes over ranks, max elapsed over ranks) via two all-reduces.

    `dist` is torch.distributed (initialised) or None for a single process."""
    if dist is None:
        return float(logical_bytes), float(elapsed_s)
    import torch
    t = torch.tensor([float(logical_bytes)], dtype=torch.float64, device=device)
    e = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(t.item()), float(e.item())


def job_rate_gibs(total_bytes, max_elapsed_s):
    """Whole-job GiB/s: the job finishes when its slowest rank does."""
    return total_bytes / max_elapsed_s / 2**30 if max_elapsed_s > 0 else 0.0
