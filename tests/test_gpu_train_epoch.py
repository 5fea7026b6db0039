"""The native epoch loop (asrx.train.train_epoch_native: train.py:6-55 on the Trainer, with the cross-entropy
kernel's fused argmax and one host synchronisation per epoch) against the reference-semantics mirror
(asrx.train.train_epoch, which runs the model's autograd path, torch's CrossEntropyLoss and logits.argmax)."""
import pytest
import torch

from oracle.ref_model import CONFIGS, det_params, synthetic_batch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def build(name):
    import asrx
    cfg = CONFIGS[name]["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    return m.to(dev).train(), cfg


def loader(name, n):
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    out = []
    for i in range(n):
        s, t, k = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=300 + i)
        out.append({"spectrum": s, "text": t, "mask": k})
    return out


@pytest.mark.parametrize("name", ["c1", "g64"])
def test_native_epoch_matches_reference_loop(name):
    """lr = 0 (the weights stay put): every batch's predictions equal the mirror's `logits.argmax(-1)` exactly and
    the epoch's mean loss matches torch's CrossEntropyLoss (fp32, 1e-5)."""
    from asrx.train import Trainer, train_epoch, train_epoch_native
    data = loader(name, 3)
    m1, _ = build(name)
    opt = torch.optim.SGD(m1.parameters(), lr=0.0)
    ref_metrics, ref_preds, ref_targets = train_epoch(m1, data, torch.nn.CrossEntropyLoss(), opt, dev)
    m2, _ = build(name)
    tr = Trainer(m2, lr=0.0, preds=True)
    metrics, preds, targets = train_epoch_native(tr, data)
    assert len(preds) == len(ref_preds) == 3
    for a, b in zip(preds, ref_preds):
        assert a.shape == b.shape and torch.equal(a, b.to(a.dtype))
    for a, b in zip(targets, ref_targets):
        assert torch.equal(a, b)
    assert abs(metrics["Train Loss"] - ref_metrics["Train Loss"]) <= 1e-5 * abs(ref_metrics["Train Loss"])


def test_native_epoch_graph_equals_eager():
    """5 AdamW steps with the shifted decoder inputs as a 4th captured buffer: the HIP-graph epoch (eager warm-up,
    capture, replays) and the eager epoch give identical losses, predictions and weights."""
    from asrx.train import Trainer, train_epoch_native
    data = loader("c1", 5)
    out = []
    for graph in (False, True):
        m, _ = build("c1")
        tr = Trainer(m, lr=1e-3, graph=graph, preds=True)
        metrics, preds, _ = train_epoch_native(tr, data)
        assert (tr._cap is not None) == graph
        out.append((metrics, preds, tr.store.flat.clone()))
    assert out[0][0] == out[1][0]
    assert all(torch.equal(a, b) for a, b in zip(out[0][1], out[1][1]))
    assert torch.equal(out[0][2], out[1][2])


def test_shift_inputs_is_the_reference_index_put():
    """train.py:22-25 as written (batch-coupled: every row's columns mask.sum(-1) - 1 take the last column)."""
    from asrx.train import shift_inputs
    text = torch.arange(2 * 6, device=dev).view(2, 6)
    mask = torch.tensor([[1, 1, 1, 0, 0, 0], [1, 1, 1, 1, 1, 0]], device=dev)
    inp, mk = shift_inputs(text, mask)
    ref_t = text.clone()
    ref_t[:, torch.tensor([2, 4], device=dev)] = ref_t[:, -1]
    assert torch.equal(inp, ref_t)
    assert torch.equal(text, torch.arange(12, device=dev).view(2, 6))   # the caller's tensors are not modified
    assert mk[:, 2].tolist() == [0, 0] and mk[:, 4].tolist() == [0, 0]
