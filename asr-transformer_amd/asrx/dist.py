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
    """Sum-all-reduce of a flat gradient buffer in buckets.

    Overlap with the backward: the backward calls `ready(start, end)` as soon as the gradients of a contiguous
    element range of the flat buffer are final (the decoder's, then the upper encoder layers'); that range is
    all-reduced asynchronously (RCCL runs on its own stream, ordered after the compute already queued) while
    the backward continues.  `finish()` / `__call__()` reduces every range not yet issued and waits for all."""

    def __init__(self, flat_grad, group=None, bucket_mb=64, allreduce_fn=None):
        self.group = group
        self.flat = flat_grad
        self.bucket_elems = max(1, int(bucket_mb * 2 ** 20) // 4)
        self.buckets = bucket_views(flat_grad, self.bucket_elems)
        self.allreduce_fn = allreduce_fn  # injectable for CPU tests (fake backend)
        self._issued = []                 # (start, end) ranges already issued this step
        self._works = []

    @property
    def world(self):
        if self.allreduce_fn is not None:
            return getattr(self.allreduce_fn, "world", 1)
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    @property
    def active(self):
        return self.allreduce_fn is not None or (dist.is_initialized() and dist.get_world_size(self.group) > 1)

    def _issue(self, view):
        if self.allreduce_fn is not None:
            self.allreduce_fn(view)
        else:
            self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def ready(self, start, end):
        """Gradients in flat[start:end] are final: start their all-reduce now (in buckets)."""
        if not self.active or end <= start:
            return
        self._issued.append((start, end))
        for b in bucket_views(self.flat[start:end], self.bucket_elems):
            self._issue(b)

    def finish(self):
        if not self.active:
            self._issued = []
            return
        # the complement of the issued ranges, highest addresses first (those gradients finished first)
        gaps, pos = [], 0
        for a, b in sorted(self._issued):
            if a > pos:
                gaps.append((pos, a))
            pos = max(pos, b)
        if pos < self.flat.numel():
            gaps.append((pos, self.flat.numel()))
        for a, b in reversed(gaps):
            for v in reversed(bucket_views(self.flat[a:b], self.bucket_elems)):
                self._issue(v)
        for w in self._works:
            w.wait()
        self._works = []
        self._issued = []

    def __call__(self):
        self.finish()
