"""Data-parallel gradient exchange: one flat fp32 gradient buffer, all-reduced in contiguous buckets over
RCCL (torch.distributed backend "nccl" on ROCm; xGMI between the GPUs of a node).  No per-parameter copies:
buckets are views of the flat buffer.  The 1/world average is folded into the optimizer's grad scale.

Wire formats (ASRX_DP_WIRE or GradAllReduce(wire=...)):
  "fp32" — dist.all_reduce of the fp32 bucket (RCCL ring/tree, sums in fp32).
  "bf16" — half the bytes on xGMI with the sum still in fp32: the bucket is cast to bf16 and split into `world`
           chunks; an all-to-all hands rank r every peer's copy of chunk r; asrx_sum_chunks_bf16 sums them in fp32
           and rounds once; an all-gather of the reduced bf16 chunks and a cast back fill the fp32 bucket.  (RCCL's
           own bf16 all-reduce would round after every one of its world - 1 additions.)  Per-element error: one
           bf16 rounding of each rank's gradient and one of the sum (relative ~2^-8).

The reference has no multi-device code; the step semantics it defines are train.py:16-35
per batch — DP averages per-shard mean losses, which equals the global mean for equal token counts per shard.
"""
import os
from contextlib import nullcontext as _nullctx

import torch
import torch.distributed as dist

WIRE = os.environ.get("ASRX_DP_WIRE", "fp32")
# a one-rank process group still exchanges its gradients (RCCL calls, segmented graph replay, exposed-time events):
# the single-GPU rehearsal of the multi-GPU step path (bench.py with ASRX_DP_REHEARSE=1)
FORCE = os.environ.get("ASRX_DP_FORCE", "0") == "1"


def _cast(src, dst):
    """dtype conversion of a bucket: the native kernel for device tensors (the product: flat grads live on the GPU);
    torch's copy only for the CPU tensors of the gloo tests of this host logic."""
    if src.is_cuda:
        from . import kernels as K
        K.cast(src, dst)
    else:
        dst.copy_(src)


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

    def __init__(self, flat_grad, group=None, bucket_mb=64, allreduce_fn=None, wire=None, chunk_sum=None):
        self.group = group
        self.flat = flat_grad
        self.bucket_elems = max(1, int(bucket_mb * 2 ** 20) // 4)
        self.buckets = bucket_views(flat_grad, self.bucket_elems)
        self.allreduce_fn = allreduce_fn  # injectable for CPU tests (fake backend)
        self.wire = WIRE if wire is None else wire
        if self.wire not in ("fp32", "bf16"):
            raise ValueError(f"asrx.dist: unknown gradient wire format {self.wire!r}")
        # the fp32 sum of the bf16 wire: the native kernel; injectable for the CPU (gloo) tests of this host logic
        self.chunk_sum = chunk_sum
        self._issued = []                 # (start, end) ranges already issued this step
        self._works = []
        self._post = []                   # bf16 wire: (bucket view, gathered bf16, work) to copy back after wait

    @property
    def world(self):
        if self.allreduce_fn is not None:
            return getattr(self.allreduce_fn, "world", 1)
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    @property
    def active(self):
        return self.allreduce_fn is not None or (dist.is_initialized() and
                                                 (FORCE or dist.get_world_size(self.group) > 1))

    def _issue(self, view):
        if self.allreduce_fn is not None:
            self.allreduce_fn(view)
        elif self.wire == "bf16":
            self._issue_bf16(view)
        else:
            self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def _side(self, device):
        """The bf16 wire's own stream (device tensors only): its cast, all-to-all wait, chunk sum and all-gather
        issue there, so the compute stream does not wait for the all-to-all between backward segments."""
        if device.type != "cuda":
            return None
        if getattr(self, "_side_stream", None) is None:
            self._side_stream = torch.cuda.Stream(device=device)
        return self._side_stream

    def _issue_bf16(self, view):
        """Reduce-scatter by all-to-all on bf16 chunks, fp32 sum of the W copies, all-gather of the bf16 sums.
        On a side stream that first waits for the compute stream (the released gradients are final there): the
        all-to-all's wait and the sum are dependencies of that stream only, and finish() joins the compute stream
        to the all-gather before the cast back."""
        W = dist.get_world_size(self.group)
        n = view.numel()
        c = -(-n // W)
        side = self._side(view.device)
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(view.device))
        with torch.cuda.stream(side) if side is not None else _nullctx():
            send = torch.empty(W * c, dtype=torch.bfloat16, device=view.device)   # the padding past n is summed
            _cast(view, send[:n])                                                   # but never copied back
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.group, async_op=True).wait()
            mine = torch.empty(c, dtype=torch.bfloat16, device=view.device)
            if self.chunk_sum is not None:
                self.chunk_sum(recv, W, c, mine)
            else:
                from . import kernels as K
                K.sum_chunks_bf16(recv, W, c, mine)
            full = torch.empty(W * c, dtype=torch.bfloat16, device=view.device)
            work = dist.all_gather_into_tensor(full, mine, group=self.group, async_op=True)
        self._post.append((view, full, work, (send, recv, mine)))

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
        for view, full, work, _bufs in self._post:   # (the side stream's buffers live until here)
            work.wait()
            if full.is_cuda:
                # `full` was allocated on the side stream but is read here on the compute stream: tell the caching
                # allocator, so the block is not handed to a later side-stream allocation before this cast has run
                # (ordering-independent of _issue_bf16's wait_stream)
                full.record_stream(torch.cuda.current_stream(full.device))
            _cast(full[:view.numel()], view)
        self._works = []
        self._post = []
        self._issued = []

    def __call__(self):
        self.finish()
