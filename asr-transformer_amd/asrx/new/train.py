"""The `new/` family's training loop semantics (modules/Transformer/new/train.py), on libasrx.so:

* `train_epoch(model, data_loader, tokenizer, loss_function, optimizer, scheduler, device)` — new/train.py:6-55: per
  batch zero_grad -> forward -> argmax + decode -> loss -> backward -> `clip_grad_norm_(params, 1.0)` ->
  optimizer.step() -> scheduler.step(); the epoch metrics (mean loss, 1 - mean WER, sentence accuracy) and the last
  decoded sentence.  The clip is the native global-norm kernel below (no per-tensor host loop, no host sync).
* `eval_epoch(model, data_loader, tokenizer, loss_function, device)` — new/train.py:58-103: greedy `evaluate`, then
  `remove_after_eos` (native), decode, loss.
* `remove_after_eos(pred, logits, eoses, eos_token)` — new/train.py:106-112, its quirk kept: the one-hot row written
  after the EOS marks index `eoses[i]` (the EOS position), not the EOS token.
* `word_error_rate(preds, targets)` — torchmetrics.functional.word_error_rate (new/train.py:2, not installed here):
  total word-level edit distance / total reference words over the batch.
The tokenizer, the loss function, the optimizer and the scheduler are the caller's (as in the reference)."""
import torch

from .. import kernels as K

_CLIP_PARTS = 256


def _spans(params):
    """Device table {address, numel} of the fp32 gradients of `params` (cached per address set)."""
    grads = [p.grad for p in params if p.grad is not None]
    for g in grads:
        if g.dtype != torch.float32 or not g.is_contiguous() or not g.is_cuda:
            raise TypeError("asrx.new.train.clip_grad_norm_: contiguous fp32 CUDA gradients only")
    key = tuple((g.data_ptr(), g.numel()) for g in grads)
    hit = _spans.cache.get(key)
    if hit is None:
        import numpy as np
        dev = grads[0].device if grads else torch.device("cuda")
        hit = torch.empty(max(1, len(key)), 2, dtype=torch.int64, device=dev)
        if key:   # (through kernel arguments, asrx_upload: no host synchronisation when the .grad tensors are new)
            K.upload(hit, np.array(key, dtype=np.int64))
        _spans.cache = {key: hit}   # (one entry: the parameters of one model are the usual case)
    return hit, len(key)


_spans.cache = {}


def clip_grad_norm_(parameters, max_norm):
    """torch.nn.utils.clip_grad_norm_(parameters, max_norm) with norm_type 2 (new/train.py:31): every gradient times
    min(max_norm / (total_norm + 1e-6), 1).  Returns the total norm as a device scalar (asrx_clip_grad_norm)."""
    params = [parameters] if isinstance(parameters, torch.Tensor) else list(parameters)
    table, count = _spans(params)
    dev = table.device
    part = torch.empty(_CLIP_PARTS, dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    if count == 0:
        return torch.zeros((), device=dev)
    K.call("asrx_clip_grad_norm", table.data_ptr(), count, float(max_norm), part.data_ptr(), _CLIP_PARTS,
           out.data_ptr(), K.stream())
    return out[0]


def remove_after_eos(pred, logits, eoses, eos_token):
    """new/train.py:106-112 in place on the device (asrx_remove_after_eos); returns (pred, logits)."""
    if not (pred.is_cuda and logits.is_cuda and pred.dtype == torch.int64 and logits.dtype == torch.float32
            and pred.is_contiguous() and logits.is_contiguous()):
        raise TypeError("asrx.new.train.remove_after_eos: contiguous int64 pred and fp32 logits on the GPU")
    B, lp = pred.shape
    _, ll, v = logits.shape
    # the reference indexes eos[eoses[i]] (a vocab-sized row): an index outside [-v, v) raises IndexError there, a
    # negative one counts from the end of the row (and of the pred / logits rows for the slices)
    # (the kernel trusted eoses.)  Host-side positions are checked here; device-side ones are trusted, as
    # checking them would cost a host synchronisation per batch — Transformer.evaluate produces them in [0, steps).
    if not eoses.is_cuda:
        ec = eoses.detach().to(torch.int64)
        if ec.numel() and (int(ec.min()) < -v or int(ec.max()) >= v):
            raise IndexError(f"asrx.new.train.remove_after_eos: an EOS position outside [-{v}, {v})")
        if ec.numel() and int(ec.min()) < 0:   # Python slicing of pred[i, e:] / logits[i, e:] and eos[e] for e < 0
            raise NotImplementedError("asrx.new.train.remove_after_eos: negative EOS positions")
    e = eoses.to(device=pred.device, dtype=torch.int64).contiguous()
    K.call("asrx_remove_after_eos", pred.data_ptr(), B, lp, logits.data_ptr(), ll, v, e.data_ptr(), int(eos_token),
           K.stream())
    return pred, logits


def _edit_distance(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def word_error_rate(preds, targets):
    """torchmetrics.functional.word_error_rate: sum of word-level edit distances / sum of reference word counts
    (a tensor, as torchmetrics returns)."""
    if isinstance(preds, str):
        preds = [preds]
    if isinstance(targets, str):
        targets = [targets]
    errors = total = 0
    for p, t in zip(preds, targets):
        pw, tw = p.split(), t.split()
        errors += _edit_distance(pw, tw)
        total += len(tw)
    # as tensors, like torchmetrics: references without words give 0 / 0 = nan (or x / 0 = inf), not 0
    return torch.tensor(float(errors)) / torch.tensor(float(total))


def _to(batch, device):
    for k in ("encoded_text", "spectre", "spectrogram_len", "text_len", "true_text"):
        batch[k] = batch[k].to(device)


def _metrics(preds, targets, prefix):
    acc_t, wer = 0.0, 0.0
    for b in range(len(preds)):
        acc = sum(int(p == t) for p, t in zip(preds[b], targets[b])) / len(preds[b])
        wer += float(word_error_rate(preds[b], targets[b]))
        acc_t += acc
    n = len(preds)
    return {f"{prefix} Word Accuracy": 1 - wer / n, f"{prefix} Accuracy": acc_t / n}


def train_epoch(model, data_loader, tokenizer, loss_function, optimizer, scheduler, device):
    """new/train.py:6-55 (see the module docstring).  Returns (metrics, the last decoded prediction)."""
    model.to(device)
    model.train()
    total, preds, targets = 0.0, [], []
    params = [p for p in model.parameters()]
    for batch in data_loader:
        _to(batch, device)
        optimizer.zero_grad()
        logits = model(batch)
        pred = tokenizer.batch_decode(logits.argmax(dim=-1).to("cpu"), skip_special_tokens=True)
        preds.append(pred)
        targets.append(batch["text"])
        loss = loss_function(logits.transpose(1, 2), batch["true_text"])
        total += loss.item()
        loss.backward()
        clip_grad_norm_(params, 1.0)
        optimizer.step()
        scheduler.step()
    m = {"Train Loss": total / len(preds)}
    m.update(_metrics(preds, targets, "Train"))
    return m, preds[-1][-1]


def eval_epoch(model, data_loader, tokenizer, loss_function, device):
    """new/train.py:58-103.  Returns (metrics, the last decoded prediction)."""
    model.to(device)
    model.eval()
    total, preds, targets = 0.0, [], []
    for batch in data_loader:
        _to(batch, device)
        with torch.no_grad():
            pred, logits, eoses = model.evaluate(batch)
            pred = pred.to(torch.int64).contiguous()
            logits = logits.float().contiguous()
            pred, logits = remove_after_eos(pred, logits, eoses, tokenizer.eos_token_id)
            preds.append(tokenizer.batch_decode(pred.to("cpu"), skip_special_tokens=True))
            targets.append(batch["text"])
        loss = loss_function(logits.transpose(1, 2), batch["true_text"])
        total += loss.item()
    m = {"Val Loss": total / len(preds)}
    m.update(_metrics(preds, targets, "Val"))
    return m, preds[-1][-1]
