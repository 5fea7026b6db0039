"""Data-parallel gradient exchange: one flat fp32 gradient buffer, all-reduced in contiguous buckets over
RCCL (torch.distributed backend "nccl" on ROCm; xGMI between the GPUs of a node).  No per-parameter copies:
buckets are views of the flat buffer.  The 1/world average is folded into the optimizer's grad scale.

The reference has no multi-device code; the step semantics it defines are train.py:16-35
per batch — DP averages per-shard mean losses, which equals the global mean for equal token counts per shard.
"""
import torch
import torch.distributed as dist


def bucket_views(flat, bucket_elems):
    n = flat.numel()
    out = []
    o = 0
    while o < n:
        e = min(n, o + bucket_elems)
        out.append(flat[o:e])
        o = e
    return out


class GradAllReduce:
    """Sum-all-reduce of a flat gradient buffer in buckets (reverse order: the last-produced gradients —
    front-end/encoder input side — are issued last, so buckets complete roughly as backward produces them)."""

    def __init__(self, flat_grad, group=None, bucket_mb=64, allreduce_fn=None):
        self.group = group
        self.buckets = bucket_views(flat_grad, max(1, int(bucket_mb * 2 ** 20) // 4))
        self.allreduce_fn = allreduce_fn  # injectable for CPU tests (fake backend)

    @property
    def world(self):
        if self.allreduce_fn is not None:
            return getattr(self.allreduce_fn, "world", 1)
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def __call__(self):
        if self.allreduce_fn is not None:
            for b in reversed(self.buckets):
                self.allreduce_fn(b)
            return
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        works = [dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for b in reversed(self.buckets)]
        for w in works:
            w.wait()
