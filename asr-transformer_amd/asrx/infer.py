"""Inference forwards replayed from HIP graphs.

An eager asrx forward is a few hundred native launches, each paying ~10 µs of Python/ctypes enqueue: for the
smaller configurations (c2: d_model 256, B=32) that host time exceeds the GPU time.  `GraphedForward` captures
`model(spectrum, text, mask)` once per input shape (model.eval(), no autograd) and afterwards replays the graph
with the new inputs copied into the captured buffers — the forward's launches then cost one graph launch.  The
returned logits are the captured output tensor, overwritten by the next call (copy it to keep it).  Same numerics
as the eager forward: the same kernels run on the same buffers' contents.
"""
import torch


class GraphedForward:
    """callable(spectrum, text, mask) -> logits (B, L, V), as model.forward (model.py:194-198)."""

    def __init__(self, model):
        self.model = model
        self._graphs = {}

    @staticmethod
    def _key(*xs):
        return tuple((tuple(x.shape), x.dtype) for x in xs)

    def __call__(self, spectrum, text, mask):
        if self.model.training:
            raise RuntimeError("asrx.infer.GraphedForward replays inference forwards: call model.eval() first")
        key = self._key(spectrum, text, mask)
        ent = self._graphs.get(key)
        if ent is None:
            ent = self._graphs[key] = self._capture(spectrum, text, mask)
        graph, ins, out = ent
        for dst, src in zip(ins, (spectrum, text, mask)):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        graph.replay()
        return out

    def _capture(self, spectrum, text, mask):
        dev = next(self.model.parameters()).device
        ins = tuple(x.to(dev).clone() for x in (spectrum, text, mask))
        with torch.no_grad():
            self.model(*ins)                   # warm-up: flat store, kernel objects, allocator
            torch.cuda.synchronize(dev)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self.model(*ins)
        torch.cuda.synchronize(dev)
        return graph, ins, out
