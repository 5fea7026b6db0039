"""The `new/` family's training-loop semantics (asrx.new.train, for modules/Transformer/new/train.py):
word error rate (CPU), the native global-norm clip against torch.nn.utils.clip_grad_norm_, remove_after_eos against a
restatement of new/train.py:106-112, and one train / eval epoch of a small asrx.new model (GPU).

Tolerances: clip — total norm <= 1e-5 relative (the sum runs in another order than torch's norm of per-tensor norms),
clipped gradients <= 2e-6 relative; unclipped (coefficient 1) gradients bit-identical; remove_after_eos exact."""
import pytest
import torch


def test_word_error_rate_matches_the_torchmetrics_definition():
    from asrx.new.train import word_error_rate
    # total edits / total reference words over the batch (not a mean of per-sentence rates)
    assert float(word_error_rate(["a b c", "d"], ["a x c", "d e f"])) == pytest.approx(3 / 6)
    assert float(word_error_rate("the cat sat", "the cat sat")) == 0.0
    assert float(word_error_rate(["one two three"], ["one three"])) == pytest.approx(1 / 2)   # one insertion
    assert float(word_error_rate([""], ["a b"])) == pytest.approx(1.0)
    import math
    assert math.isnan(float(word_error_rate([""], [""])))         # torchmetrics' tensor 0 / 0
    assert math.isinf(float(word_error_rate(["a"], [""])))        # x / 0


gpu = pytest.mark.gpu


@pytest.fixture
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _grads(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    flat = torch.randn(300001, device="cuda", generator=g)
    ps = []
    # whole tensors and views at offsets that are not 16-B aligned (the scalar path), sizes around the chunk size
    for off, n in [(0, 1), (1, 7), (8, 4096), (4104, 4097), (8201, 100000), (108201, 12345), (120546, 179455)]:
        p = torch.nn.Parameter(torch.zeros(n, device="cuda"))
        p.grad = flat[off:off + n]
        ps.append(p)
    return ps


@gpu
@pytest.mark.parametrize("max_norm", [1.0, 1e9])
def test_clip_grad_norm_matches_torch(_need_gpu, max_norm):
    from asrx.new.train import clip_grad_norm_
    a, b = _grads(3), _grads(3)
    ref = torch.nn.utils.clip_grad_norm_(a, max_norm)
    got = clip_grad_norm_(b, max_norm)
    torch.cuda.synchronize()
    assert abs(float(got) - float(ref)) <= 1e-5 * float(ref)
    for pa, pb in zip(a, b):
        if max_norm > 1e8:
            assert torch.equal(pa.grad, pb.grad)   # coefficient 1: x 1.0 exactly
        else:
            assert float((pa.grad - pb.grad).abs().max()) <= 2e-6 * float(pa.grad.abs().max()) + 1e-30


@gpu
def test_remove_after_eos_matches_the_reference(_need_gpu):
    from asrx.new.train import remove_after_eos
    g = torch.Generator(device="cuda").manual_seed(5)
    B, L, V = 5, 9, 13
    pred = torch.randint(0, V, (B, L + 1), device="cuda", generator=g)
    logits = torch.randn(B, L, V, device="cuda", generator=g)
    eoses = torch.tensor([0, 3, 8, 4, 2])
    rp, rl = pred.clone().cpu(), logits.clone().cpu()
    for i in range(eoses.shape[0]):          # new/train.py:107-111, as written
        rp[i, eoses[i]:] = 2
        eos = torch.zeros((rl.shape[2]))
        eos[eoses[i]] = 1
        rl[i, eoses[i]:] = eos
    p2, l2 = remove_after_eos(pred, logits, eoses, 2)
    torch.cuda.synchronize()
    assert torch.equal(p2.cpu(), rp) and torch.equal(l2.cpu(), rl)


class _Tok:
    eos_token_id = 2

    def batch_decode(self, ids, skip_special_tokens=True):
        return [" ".join(str(int(t)) for t in row if not (skip_special_tokens and int(t) < 5)) for row in ids]


@gpu
def test_new_train_and_eval_epoch_run_on_the_native_path(_need_gpu):
    import asrx.new
    from oracle import ref_model_new as N
    c = N.NEW_CONFIGS["new_micro"]
    m = asrx.new.Transformer(c.vocab_size, c.n_mels, c.enc_seq_len, c.dec_seq_len, c.hidden_dim, c.n_enc, c.n_dec,
                             c.n_heads, c.ff_dim, "cuda", dropout=0.1, sr=c.sr, n_fft=c.n_fft, padding_idx=c.pad_id,
                             eos_token=c.eos_id, bos_token=c.bos_id).cuda()
    tok = _Tok()
    loader = []
    for s in range(3):
        spectre, lens, text = N.synthetic_batch(c, 4, seed=10 + s)
        true = torch.full_like(text, c.eos_id)
        true[:, :-1] = text[:, 1:]
        loader.append({"spectre": spectre, "spectrogram_len": lens, "encoded_text": text, "text_len": lens,
                       "true_text": true, "text": tok.batch_decode(true)})
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.9)
    before = [p.detach().clone() for p in m.parameters()]
    metrics, last = asrx.new.train_epoch(m, loader, tok, torch.nn.CrossEntropyLoss(), opt, sched, "cuda")
    assert set(metrics) == {"Train Loss", "Train Word Accuracy", "Train Accuracy"}
    assert metrics["Train Loss"] == metrics["Train Loss"] and metrics["Train Loss"] > 0
    assert isinstance(last, str)
    assert sched.last_epoch == 3
    assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
    # after the epoch's last clip, the gradients' global norm is <= 1 (+ rounding)
    norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in m.parameters() if p.grad is not None))
    assert float(norm) <= 1.0 + 1e-5
    vm, vlast = asrx.new.eval_epoch(m, loader, tok, torch.nn.CrossEntropyLoss(), "cuda")
    assert set(vm) == {"Val Loss", "Val Word Accuracy", "Val Accuracy"}
    assert vm["Val Loss"] == vm["Val Loss"] and isinstance(vlast, str)
