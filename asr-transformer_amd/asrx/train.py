"""Training / evaluation loops.

`train_epoch` / `eval_epoch` mirror modules/Transformer/train.py:6-108 (same arguments, same batch dict keys,
same metrics dict) for drop-in use with any torch optimizer and loss.

`Trainer` is the MI355X-native step: forward -> fused cross-entropy kernel -> explicit backward -> RCCL
bucketed gradient all-reduce -> fused AdamW over the flat parameter buffer (which also refreshes the bf16
operand copy).  No autograd graph, no per-parameter launches.  After two eager steps the step is captured as
HIP graph(s) and replayed (about 700 launches otherwise cost ~13 ms of Python/ctypes enqueue per step, as much as
the GPU work): per-step values reach the replay through device memory (dropout seed offset, Adam lr / bias
corrections), new batches are copied into the captured input buffers.  With a multi-GPU reducer the backward
is captured in segments that end where gradient ranges become final; the RCCL all-reduce of each range is
issued between segment replays, so it still overlaps the rest of the backward.
"""
import os

import torch

from . import kernels as K
from .blocks import FreshGrads
from .dist import GradAllReduce
from .functions import get_store, make_ctx, model_backward, model_forward

# weight gradients whose only writer is one weight-gradient GEMM are not zeroed before the backward: that GEMM
# writes them with beta = 0 (blocks.FreshGrads).  ASRX_FRESH_GRADS=0 zeroes the whole buffer instead (A/B).
FRESH_GRADS = os.environ.get("ASRX_FRESH_GRADS", "1") == "1"
# capture the training step as HIP graph(s) after the eager warm-up steps (ASRX_GRAPH=0: eager steps, A/B)
GRAPH = os.environ.get("ASRX_GRAPH", "1") == "1"
GRAPH_WARMUP = 2
# multi-GPU, ASRX_DP_EARLY_ADAM=1: AdamW of the ranges all-reduced mid-backward runs on a side stream as soon as
# their all-reduces are done, beside the rest of the backward, instead of after the final all-reduce.  Off: in the
# one-rank RCCL rehearsal it was slower (14.35 / 14.26 vs 14.12 / 14.13 ms, ABAB) — the side AdamW starts right at
# the release point and takes HBM bandwidth from the HBM-bound encoder backward it runs beside
EARLY_ADAM = os.environ.get("ASRX_DP_EARLY_ADAM", "0") == "1"
# single-GPU steps: AdamW of every nn.Linear parameter fused into the grouped weight-gradient launch, the rest by
# one span-table launch (ASRX_FUSED_ADAM=0: the separate optimizer launch over the flat buffers)
FUSED_ADAM = os.environ.get("ASRX_FUSED_ADAM", "1") == "1"
ADAM_SPAN = 8192   # elements per workgroup of the residual span-table launch
ZERO_SPAN = 16384  # elements per workgroup of the per-step gradient zeroing (asrx_zero_spans)


def _aligned_spans(spans, n, q=4):
    """Union of [a, b) spans shrunk to multiples of q elements (16-B aligned fp32 / 8-B aligned bf16 views)."""
    out = []
    for a, b in sorted(spans):
        a, b = -(-a // q) * q, min(n, b) // q * q
        if b <= a:
            continue
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [tuple(x) for x in out]


def _complement(spans, n):
    out, pos = [], 0
    for a, b in spans:
        if a > pos:
            out.append((pos, a))
        pos = b
    if pos < n:
        out.append((pos, n))
    return out


class _Segments:
    """A training step captured as a sequence of HIP graphs sharing one memory pool, replayed in order.

    A new segment starts where (a) the backward hands finished gradient ranges to the all-reduce (`ready` +
    `boundary`: the replay issues their RCCL all-reduce between segment replays, overlapping the rest of the
    backward) or (b) the bench's kernel probe times one kernel (`split`: that kernel gets a segment of its own,
    bracketed by HIP events at replay)."""

    def __init__(self, pool):
        self.pool = pool
        self.graphs, self.after, self.timed = [], [], []
        self._pending = []
        self._begin(None)

    def _begin(self, timed):
        g = torch.cuda.CUDAGraph()
        # thread_local: another thread's query of a non-captured stream (torch's RCCL watchdog polls the events of
        # finished all-reduces) must not invalidate this capture — "global" mode turned such a poll into a failed
        # capture and an aborted process in the one-rank RCCL rehearsal
        g.capture_begin(pool=self.pool, capture_error_mode="thread_local")
        self.graphs.append(g)
        self.timed.append(timed)

    def _end(self):
        self.graphs[-1].capture_end()
        self.after.append(self._pending)
        self._pending = []

    def __call__(self, a, b):
        self._pending.append((a, b))

    def boundary(self):
        self._end()
        self._begin(None)

    def split(self, timed):
        self._end()
        self._begin(timed)

    def close(self):
        self._end()

    def replay(self, reducer):
        probe = K.PROBE
        for g, spans, timed in zip(self.graphs, self.after, self.timed):
            if timed is not None and probe is not None and probe.record(timed[0]):
                name, flops = timed
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                g.replay()
                s1.record()
                probe.events.setdefault(name, []).append((s0, s1))
                probe.flops[name] = probe.flops.get(name, 0) + flops
            else:
                g.replay()
            for a, b in spans:
                reducer.ready(a, b)


def residual_pieces(n, cover, piece=None):
    """The [start, end) ranges of a flat buffer of n elements NOT covered by the (offset, numel) ranges `cover`, cut
    into pieces of at most `piece` elements (default ADAM_SPAN).  Every parameter starts 64-aligned, so with whole
    parameters as cover the bounds are multiples of 4; others are kept exact (never rounded into a covered quad)."""
    piece = piece or ADAM_SPAN
    out = []
    for a, b in _minus(0, n, sorted(cover)):
        # exact bounds (asrx_adam_spans steps unaligned heads / tails one element at a time), inner cuts on quads
        cuts = [a] + list(range(a // 4 * 4 + piece, b, piece)) + [b]
        out += [(c0, c1) for c0, c1 in zip(cuts[:-1], cuts[1:]) if c1 > c0]
    return out


def _minus(a, b, holes, align=1):
    """[a, b) without the (offset, numel) ranges `holes` (sorted): the remaining non-empty runs, in order.  align = 4
    rounds each hole's end up to a multiple of 4 elements — for runs that feed asrx_adam, which takes 16-B aligned
    ranges only; holes that are whole parameters of the flat store (every one starts 64-aligned) then end in padding
    (ADVICE r5)."""
    out, pos = [], a
    for o, k in holes:
        if o + k <= pos or o >= b:
            continue
        if o > pos:
            out.append((pos, o))
        pos = max(pos, (o + k + align - 1) // align * align)
    if pos < b:
        out.append((pos, b))
    return out


def unused_params(model):
    """Parameters the reference's forward never uses, so they never get a gradient there (their .grad stays None and
    torch's optimizers skip them): input_encoding (model.py:173) and Encoder._norm_in (model.py:12)."""
    out = []
    for m in (getattr(model, "input_encoding", None), getattr(getattr(model, "encoder", None), "_norm_in", None)):
        if m is not None:
            out += list(m.parameters())
    return out


def wgrad_only_params(model):
    """Parameters written only by a weight-gradient GEMM: the Linear weights (incl. the packed Q/K/V and K/V
    projections and the classifier).  Biases (fused row sums accumulate), LayerNorm, embedding and conv
    parameters have accumulating writers and are zeroed each step."""
    from .layers import MHA, _Lin
    from .model import _Classifier
    out = []
    # (input_encoding is built but unused by the reference, model.py:173: no GEMM writes its gradient, so it stays in
    #  the zeroed spans instead of being drained by a torch fill every step)
    unused = {id(m) for m in (getattr(model, "input_encoding", None),) if m is not None}
    for m in model.modules():
        if id(m) in unused:
            continue
        if isinstance(m, (_Lin, _Classifier)):
            out.append(m.weight)
        elif isinstance(m, MHA):
            out += [p for p in (getattr(m, "wq", None), getattr(m, "wkv", None), getattr(m, "wqkv", None))
                    if p is not None]
    return out


def train_epoch(model, data_loader, loss_function, optimizer, device):
    """train.py:6-55 semantics, including the teacher-forcing shift of train.py:22-25 as written (a
    batch-coupled index_put)."""
    model.to(device)
    model.train()
    total = 0.0
    preds, targets = [], []
    for batch in data_loader:
        spectrum = batch["spectrum"].to(device)
        text = batch["text"].to(device)
        mask = batch["mask"].to(device)
        input_text = text.detach().clone()
        input_text[:, mask.sum(dim=-1).long() - 1] = input_text[:, -1]
        mask = mask.clone()
        mask[:, mask.sum(dim=-1).long() - 1] = mask[:, -1]
        input_text, mask = input_text[:, :-1], mask[:, :-1]
        optimizer.zero_grad()
        logits = model(spectrum, input_text, mask)
        preds.append(logits.argmax(dim=-1).to("cpu"))
        targets.append(text[:, :-1].to("cpu"))
        loss = loss_function(logits.transpose(1, 2), text[:, 1:])
        total += loss.item()
        loss.backward()
        optimizer.step()
    return {"Train Loss": total / max(1, len(data_loader))}, preds, targets


def shift_inputs(text, mask):
    """train.py:22-25 as written: the decoder input is a copy of text whose columns mask.sum(-1) - 1 (one column
    per sample, applied to EVERY row: a batch-coupled index_put) take the last column, and the mask
    the same; device ops, no host sync.  Returns (input_text, mask), both (B, L+1): the step drops the last column."""
    idx = mask.sum(dim=-1).long() - 1
    input_text = text.detach().clone()
    input_text[:, idx] = input_text[:, -1]
    mask = mask.clone()
    mask[:, idx] = mask[:, -1]
    return input_text, mask


def train_epoch_native(trainer, data_loader, device=None):
    """train_epoch (train.py:6-55) on the native step: the same shifted inputs, targets, per-step predictions
    (`logits.argmax(-1)`, here the cross-entropy kernel's fused argmax) and mean loss, but losses are summed and
    predictions kept on the device — ONE host synchronisation per epoch instead of two per step (`.item()`,
    `.to('cpu')`; train.py:30,33).  trainer: an asrx.train.Trainer built with preds=True.
    Returns ({"Train Loss": mean}, preds, targets) like train_epoch (preds / targets: CPU int64 (B, L))."""
    if not trainer.want_preds:
        raise ValueError("train_epoch_native needs Trainer(..., preds=True)")
    dev = torch.device(device) if device is not None else trainer.store.flat.device
    trainer.model.train()
    total = torch.zeros((), dtype=torch.float32, device=dev)
    preds, targets, n = [], [], 0
    for batch in data_loader:
        spectrum = batch["spectrum"].to(dev)
        text = batch["text"].to(dev)
        mask = batch["mask"].to(dev)
        input_text, mask = shift_inputs(text, mask)
        loss = trainer.step(spectrum, text, mask, input_text=input_text)
        total += loss.reshape(())                      # before the next step overwrites a replayed graph's output
        B, L = text.shape[0], text.shape[1] - 1
        preds.append(trainer.last_preds.view(B, L).clone())
        targets.append(text[:, :-1])
        n += 1
    torch.cuda.synchronize(dev)
    preds = [p.cpu() for p in preds]
    targets = [t.cpu() for t in targets]
    return {"Train Loss": float(total) / max(1, n)}, preds, targets


def eval_epoch(model, data_loader, eos_token_id, bos_token_id, loss_function, device):
    """train.py:58-108: greedy decode per batch (Transformer.evaluate), logits padded/truncated to the
    target length, CE loss averaged over batches."""
    model.to(device)
    model.eval()
    total = 0.0
    preds, targets = [], []
    with torch.no_grad():
        for batch in data_loader:
            spectrum = batch["spectrum"].to(device)
            text = batch["text"].to(device)
            text_in = torch.full((text.shape[0], 1), bos_token_id, dtype=torch.int32).to(device)
            pred, logits = model.evaluate(spectrum, text_in)
            text = text[:, 1:]
            for i in range(len(logits)):
                if logits[i].shape[0] > text.shape[1]:
                    logits[i] = logits[i][:text.shape[1]]
                else:
                    logits[i] = torch.cat((logits[i], torch.zeros((text.shape[1] - logits[i].shape[0],
                                                                   logits[i].shape[1]), device=logits[i].device)),
                                          dim=0)
            logits = torch.stack(logits, dim=0)
            preds.append(pred.to("cpu"))
            targets.append(text.to("cpu"))
            loss = loss_function(logits.transpose(1, 2), text)
            total += loss.item()
    return {"Val Loss": total / max(1, len(data_loader))}, preds[-1][-1]


class Trainer:
    """Native data-parallel training step for an asrx.Transformer."""

    def __init__(self, model, lr=1e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=0.0, decoupled=True,
                 ignore_index=-100, group=None, bucket_mb=64, allreduce_fn=None, graph=None, wire=None, preds=False):
        self.model = model
        self.store = get_store(model)
        self.m = torch.zeros_like(self.store.flat)
        self.v = torch.zeros_like(self.store.flat)
        self.lr, self.betas, self.eps, self.wd, self.decoupled = lr, betas, eps, weight_decay, decoupled
        self.ignore_index = ignore_index
        self.step_count = 0
        self.reducer = GradAllReduce(self.store.grad, group=group, bucket_mb=bucket_mb, allreduce_fn=allreduce_fn,
                                     wire=wire)
        self.store.refresh_shadow(force=True)
        self._wonly = wgrad_only_params(model) if FRESH_GRADS else []
        self.graph = GRAPH if graph is None else bool(graph)
        self._cap = None        # captured step of the current input shape: (segments, static inputs, loss, preds)
        self._caps = {}         # every captured step, keyed by input shapes (a smaller last batch keeps its own graph)
        self._eager_keys = set()   # input shapes that have run one eager step (captured only after one)
        self._hyp = torch.zeros(3, dtype=torch.float32, device=self.store.flat.device)
        self.ar_events = None   # list -> record the exposed all-reduce time of each step (_finish)
        self._adam_side = None  # multi-GPU early AdamW stream (_reduce_and_adam)
        # preds=True: the cross-entropy kernel also writes each row's argmax over the V classes (train.py:29,
        # `logits.argmax(-1)`, fused into the loss pass) into last_preds (int64 [B*L], device; in graph mode the
        # captured buffer, overwritten by the next step)
        self.want_preds = bool(preds)
        self.last_preds = None
        self._cover = None       # flat-gradient ranges whose AdamW the last backward ran fused (None: none)
        self._rspans = {}        # residual-range tables by cover
        self._fuse_next = False  # the next forward_backward fuses AdamW (set by step(), which owns the optimizer)
        # parameters the reference never gives a gradient (input_encoding, model.py:173; Encoder._norm_in, model.py:12):
        # torch's AdamW skips a parameter whose grad is None, so every AdamW launch here leaves their ranges alone
        # (a zero-gradient step would still apply weight decay to them)
        self._frozen = sorted((self.store.offset(p), p.numel()) for p in unused_params(model)
                              if self.store.owns(p))
        if self._wonly:   # the spans of everything else, zeroed each step by one asrx_zero_spans launch
            n, spans, pos = self.store.grad.numel(), [], 0
            for o, k in sorted((self.store.offset(p), p.numel()) for p in self._wonly):
                if o > pos:
                    spans.append((pos, o))
                pos = max(pos, o + k)
            if pos < n:
                spans.append((pos, n))
            # (one workgroup per row of the table: long spans — the embedding, the front-end, the positional tables —
            #  cut into ZERO_SPAN pieces, round 5; a 512 KiB span on one workgroup took most of the launch's 21 us)
            spans = [(c, min(c + ZERO_SPAN, b)) for a, b in spans for c in range(a, b, ZERO_SPAN)]
            self._zero_spans = torch.tensor(spans, dtype=torch.int64).reshape(-1, 2).to(self.store.grad.device)

    def _fused_adam_ok(self):
        """AdamW fused into the grouped weight-gradient launch: single GPU (no gradient exchange before the step),
        bf16, FreshGrads, one end-of-backward flush (ASRX_FUSED_ADAM=0: the separate optimizer launch)."""
        return FUSED_ADAM and not self.reducer.active and self.model.precision == "bf16" and bool(self._wonly)

    def _residual_spans(self, cover):
        """Device [n, 2] table of the flat ranges NOT covered by the fused launch, cut into pieces of at most
        ADAM_SPAN elements (one workgroup each); cached per cover (built in the eager step that precedes a capture)."""
        key = tuple(sorted(cover))
        tab = self._rspans.get(key)
        if tab is None:
            pieces = residual_pieces(self.store.flat.numel(), sorted(key + tuple(self._frozen)))
            tab = torch.tensor(pieces, dtype=torch.int64).reshape(-1, 2).to(self.store.flat.device)
            self._rspans[key] = tab
        return tab

    def forward_backward(self, spectrum, text, mask, ready=None, capture=False, input_text=None):
        """text: (B, L+1) with BOS ... ; inputs text[:, :-1], targets text[:, 1:] (train.py:24,32).  input_text
        (optional, (B, L+1)): the decoder input instead of text (train.py:22-25 feeds a shifted copy while the
        targets stay text[:, 1:]).  ready: gradient-range hook (default: the reducer's, when multi-GPU); capture:
        building a HIP graph."""
        model = self.model
        C = make_ctx(model, model.decoder.p)
        inp = text if input_text is None else input_text
        if (text.is_cuda and text.dtype == torch.int64 and inp.dtype == torch.int64 and mask.dtype == torch.float32
                and text.stride(1) == 1 and inp.stride(1) == 1 and mask.stride(1) == 1):
            # the shifted inputs, targets and decoder mask in one native launch (no torch copies in the step)
            B, L = text.shape[0], text.shape[1] - 1
            dec_in, tgt, valid = K.step_tokens(text, inp, mask)
            spec = K.MaskSpec(1, True, valid, valid, valid.stride(0))
            logits, S = model_forward(C, model, spectrum, dec_in.view(B, L), None, spec=spec)
        else:
            logits, S = model_forward(C, model, spectrum, inp[:, :-1], mask[:, :-1])
            tgt = text[:, 1:].reshape(-1).contiguous()
        V = model.decoder._classifier.V
        loss, dl, am = K.cross_entropy(logits, V, tgt, ignore_index=self.ignore_index, want_argmax=self.want_preds)
        self.last_preds = am
        if self._wonly and C.cd == torch.bfloat16 and all(p.grad is not None for p in self.store.params):
            K.zero_spans(self.store.grad, self._zero_spans)
            C.fresh = FreshGrads(self.store, self._wonly)
        else:
            self.store.grad.zero_()
        self._cover = None
        if self._fuse_next and C.fresh is not None:
            sh = self.store.shadow
            C.adam = K.adam_desc(self.store.flat, self.m, self.v, sh, self.store.grad, self.lr, self.betas[0],
                                 self.betas[1], self.eps, self.wd, max(1, self.step_count + 1),
                                 grad_scale=1.0 / self.reducer.world, decoupled=self.decoupled, hyp=self._hyp)
        if ready is None and not capture and self.reducer.active:
            ready = self.reducer.ready
        model_backward(C, model, S, dl.to(C.cd) if dl.dtype != C.cd else dl, ready=ready)
        if C.fresh is not None:
            C.fresh.drain()
            C.fresh = None
        if C.adam is not None and C.adam_cover:
            self._cover = list(C.adam_cover)
        return loss

    def _adam(self, hyp=None, span=None):
        if span is None and self._cover is not None:   # the fused launch updated its ranges: AdamW for the rest
            sh = self.store.shadow
            K.adam_spans(self.store.flat, self.store.grad, self.m, self.v, sh, self._residual_spans(self._cover),
                         self.lr, self.betas[0], self.betas[1], self.eps, self.wd, max(1, self.step_count),
                         grad_scale=1.0 / self.reducer.world, decoupled=self.decoupled, hyp=hyp)
            return
        a0, b0 = span if span is not None else (0, self.store.flat.numel())
        for a, b in _minus(a0, b0, self._frozen, align=4):
            sh = self.store.shadow[a:b] if self.store.shadow is not None else None
            K.adam(self.store.flat[a:b], self.store.grad[a:b], self.m[a:b], self.v[a:b], sh, self.lr, self.betas[0],
                   self.betas[1], self.eps, self.wd, max(1, self.step_count), grad_scale=1.0 / self.reducer.world,
                   decoupled=self.decoupled, hyp=hyp)

    def _reduce_and_adam(self, hyp=None):
        """finish() the gradient exchange and run AdamW.  Multi-GPU over RCCL (fp32 wire): the ranges released
        mid-backward get their AdamW on a side stream that waits only for their all-reduces — each of which RCCL
        ordered after the backward's release point, so every read of those weights and gradients in this step is
        behind it — and the compute stream takes the rest after finish(), then joins the side stream."""
        red = self.reducer
        n = self.store.flat.numel()
        early = []
        if EARLY_ADAM and red.active and red.allreduce_fn is None and red.wire == "fp32" and red._issued:
            early = _aligned_spans(red._issued, n)
        if not early:
            self._finish()
            self._adam(hyp)
            return
        dev = self.store.flat.device
        if self._adam_side is None:
            self._adam_side = torch.cuda.Stream(device=dev)
        side, main = self._adam_side, torch.cuda.current_stream(dev)
        works = list(red._works)
        with torch.cuda.stream(side):
            for w in works:
                w.wait()
            for sp in early:
                self._adam(hyp, sp)
        self._finish()
        for sp in _complement(early, n):
            self._adam(hyp, sp)
        main.wait_stream(side)

    def step(self, spectrum, text, mask, input_text=None):
        """One training step (forward, CE, backward, all-reduce, AdamW).  Returns the loss as a device scalar; in
        graph mode it is the captured output tensor, overwritten by the next step.  input_text: see
        forward_backward."""
        if input_text is None:
            input_text = text
        if self.graph and self.model.precision == "bf16":
            key = self._key(spectrum, text, mask, input_text)
            self._cap = self._caps.get(key)
            # a new input shape runs one eager step first (kernel objects, allocator), then is captured and kept
            if self._cap is None and self.step_count >= GRAPH_WARMUP and key in self._eager_keys:
                self._capture(spectrum, text, mask, input_text)
                self._caps[key] = self._cap
            if self._cap is not None:
                return self._replay(spectrum, text, mask, input_text)
            self._eager_keys.add(key)
        self._fuse_next = self._fused_adam_ok()
        # this step's lr / bias corrections from the device, as in a replayed graph (and the fused launch): every
        # AdamW of the trainer takes 1/sqrt(bias_corr2) from the same device arithmetic
        K.adam_hyper(self._hyp, self.lr, self.betas[0], self.betas[1], self.step_count + 1)
        try:
            loss = self.forward_backward(spectrum, text, mask, input_text=input_text)
        finally:
            self._fuse_next = False
        self.step_count += 1
        self._reduce_and_adam(self._hyp)
        self.store.mark_shadow_fresh()
        return loss

    def _finish(self):
        """The all-reduce of whatever the backward did not release, waited for on the compute stream.  With
        `ar_events` set to a list (bench.py), HIP events bracket it on that stream: their elapsed time is the
        all-reduce time the backward did not hide (exposed), per step and rank."""
        if self.ar_events is not None and self.reducer.active:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.reducer.finish()
            e1.record()
            self.ar_events.append((e0, e1))
        else:
            self.reducer.finish()

    # ---- HIP graph mode
    @staticmethod
    def _key(*xs):
        return tuple((tuple(x.shape), x.dtype) for x in xs)

    def _capture(self, spectrum, text, mask, input_text):
        dev = self.store.flat.device
        ins = tuple(x.to(dev).clone() for x in (spectrum, text, mask, input_text))
        torch.cuda.synchronize(dev)
        pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            seg = _Segments(pool)
            K.CAPTURE = seg
            self._fuse_next = self._fused_adam_ok()
            try:
                loss = self.forward_backward(*ins[:3], ready=seg if self.reducer.active else None, capture=True,
                                             input_text=ins[3])
                if not self.reducer.active:
                    self._adam(self._hyp)
            finally:
                self._fuse_next = False
                K.CAPTURE = None
                seg.close()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self._cap = (seg, ins, loss, self.last_preds)

    def _replay(self, spectrum, text, mask, input_text):
        seg, ins, loss, preds = self._cap
        self.last_preds = preds
        for dst, src in zip(ins, (spectrum, text, mask, input_text)):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.step_count += 1
        K.set_seed_offset(self.step_count)
        K.adam_hyper(self._hyp, self.lr, self.betas[0], self.betas[1], self.step_count)
        seg.replay(self.reducer)
        if self.reducer.active:
            self._reduce_and_adam(self._hyp)
        self.store.mark_shadow_fresh()
        return loss
