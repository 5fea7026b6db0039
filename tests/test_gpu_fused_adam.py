"""AdamW fused into the grouped weight-gradient launch (asrx_gemm_grouped_xcd_adam + asrx_adam_spans for the other
parameters; asrx.train.FUSED_ADAM) against the separate optimizer launch (asrx_adam over the flat buffers):
the element update is the same code (common.h adam_elem, contraction off), so parameters, moments and the bf16
shadow must agree bit for bit after several steps — eager and HIP-graph."""
import pytest
import torch

from oracle.ref_model import CONFIGS, det_params, synthetic_batch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def build(name, dropout):
    import asrx
    cfg = CONFIGS[name]["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=dropout, precision="bf16")
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    return m.to(dev).train(), cfg


def run(name, fused, graph, steps, batch, dropout=0.0, wd=0.0, decoupled=True, wkind=None):
    import asrx.kernels as KK
    import asrx.train as T
    old, oldk = T.FUSED_ADAM, KK.WGRAD_KIND
    T.FUSED_ADAM = fused
    if wkind:
        KK.WGRAD_KIND = wkind
    try:
        m, cfg = build(name, dropout)
        spec = CONFIGS[name]
        data = []
        for i in range(steps):
            s, t, k = synthetic_batch(cfg, batch, spec["frames"], spec["text_len"] + 1, seed=300 + i)
            data.append((s.to(dev), t.to(dev), k.to(dev)))
        tr = T.Trainer(m, lr=2e-3, weight_decay=wd, decoupled=decoupled, graph=graph)
        losses = [float(tr.step(*b)) for b in data]
        torch.cuda.synchronize()
        return tr, losses
    finally:
        T.FUSED_ADAM = old
        KK.WGRAD_KIND = oldk


@pytest.mark.parametrize("wd,decoupled", [(0.0, True), (0.01, True), (0.01, False)])
def test_fused_adam_equals_separate_adam_eager(wd, decoupled, wkind="ws"):
    """c3 dimensions at B = 2 (the bench's GEMM shapes per row, the ws queue launch): 4 eager
    AdamW steps; from the second (FreshGrads) on the fused path runs, covering every nn.Linear weight and bias
    gradient."""
    ref, l0 = run("c3", False, False, 4, 2, wd=wd, decoupled=decoupled, wkind=wkind)
    tr, l1 = run("c3", True, False, 4, 2, wd=wd, decoupled=decoupled, wkind=wkind)
    assert tr._cover, "the fused launch did not run"
    assert ref._cover is None
    covered = sum(k for _, k in tr._cover)
    assert covered > 0.9 * tr.store.flat.numel(), covered       # the Linear layers: nearly every parameter
    assert l0 == l1
    for a, b in ((ref.store.flat, tr.store.flat), (ref.m, tr.m), (ref.v, tr.v), (ref.store.shadow, tr.store.shadow)):
        assert torch.equal(a, b)


def test_fused_adam_graph_equals_eager(wkind="ws"):
    """The captured step (fused launch + residual span-table AdamW, per-step hyper-parameters from the device) equals
    the eager fused step bit for bit over 5 steps (2 eager warm-up steps, capture, replays)."""
    e, l0 = run("c3", True, False, 5, 2, wkind=wkind)
    g, l1 = run("c3", True, True, 5, 2, wkind=wkind)
    assert g._cap is not None and g._cover
    assert l0 == l1
    assert torch.equal(e.store.flat, g.store.flat)
    assert torch.equal(e.m, g.m) and torch.equal(e.v, g.v)
