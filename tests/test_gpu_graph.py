"""The HIP-graph training step (asrx.train.Trainer after its eager warm-up steps) against the eager step.

Per-step values reach a replayed graph through device memory: the dropout seed offset (asrx_set_seed_offset),
the Adam lr / bias corrections (asrx_adam hyp) and the captured input buffers.  With dropout 0 every kernel is
deterministic, so graph and eager steps must agree bit for bit."""
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


def batches(cfg, spec, n, batch=None):
    out = []
    for i in range(n):
        s, t, k = synthetic_batch(cfg, batch or spec["batch"], spec["frames"], spec["text_len"] + 1, seed=100 + i)
        out.append((s.to(dev), t.to(dev), k.to(dev)))
    return out


@pytest.mark.parametrize("name", ["c1", "g64"])
def test_graph_steps_equal_eager_steps(name):
    """6 AdamW steps over changing batches: eager (graph=False) and graph (eager warm-up, capture, replays with new
    inputs copied into the captured buffers and per-step Adam bias corrections) give identical parameters."""
    from asrx.train import Trainer
    spec = CONFIGS[name]
    data = None
    params = []
    for graph in (False, True):
        m, cfg = build(name, 0.0)
        data = data or batches(cfg, spec, 6)
        tr = Trainer(m, lr=1e-3, graph=graph)
        losses = [float(tr.step(*b)) for b in data]
        torch.cuda.synchronize()
        assert (tr._cap is not None) == graph
        params.append((tr.store.flat.clone(), losses))
    assert params[0][1] == params[1][1]
    assert torch.equal(params[0][0], params[1][0])


def test_graph_dropout_masks_change_per_replay():
    """With dropout, each replay draws fresh masks (device seed offset): at lr = 0 the same batch gives a different
    loss every step, yet forward and backward of a step agree (finite gradients, repeatable given the offset)."""
    from asrx import kernels as K
    from asrx.train import Trainer
    m, cfg = build("c1", 0.1)
    spec = CONFIGS["c1"]
    (b,) = batches(cfg, spec, 1)
    tr = Trainer(m, lr=0.0, graph=True)
    losses = [float(tr.step(*b)) for _ in range(6)]
    assert tr._cap is not None
    replays = losses[2:]
    assert len(set(replays)) == len(replays), losses
    assert torch.isfinite(tr.store.grad).all()
    # the same offset reproduces the same masks
    K.set_seed_offset(4)
    seg, ins, loss = tr._cap[:3]
    K.adam_hyper(tr._hyp, 0.0, 0.9, 0.98, 4)
    seg.replay(tr.reducer)
    assert float(loss) == losses[3]
    K.set_seed_offset(0)


def test_graph_segments_with_release_path(monkeypatch):
    """Multi-GPU structure on one GPU: with a reducer the backward is captured in segments ending where gradient
    ranges become final; the injected all-reduce (doubling each range) runs between segment replays.  Graph
    replays must give the same gradients as eager steps with the same reducer (dropout 0, lr 0).  Fixed one-layer
    release groups: the default (groups sized to a round of weight-gradient tiles) keeps c2's small encoder whole."""
    from asrx import functions
    from asrx.train import Trainer
    monkeypatch.setattr(functions, "RELEASE_LAYERS", 1)
    m, cfg = build("c2", 0.0)
    spec = CONFIGS["c2"]
    (b,) = batches(cfg, spec, 1, batch=8)
    grads = []
    for graph in (False, True):
        seen = []

        def fake(view):
            seen.append(view.numel())
            view.mul_(2.0)
        tr = Trainer(m, lr=0.0, allreduce_fn=fake, graph=graph)
        for _ in range(4):
            seen.clear()
            tr.step(*b)
        torch.cuda.synchronize()
        assert (tr._cap is not None) == graph
        if graph:
            assert len(tr._cap[0].graphs) > 1
        assert len(seen) > 1
        grads.append(tr.store.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_graph_steps_keyed_by_shape():
    """Alternating input shapes (a smaller last batch every other step): each shape runs one eager step, is then
    captured once and replayed — both graphs are kept — and the 8 steps equal the eager Trainer's bit for bit."""
    from asrx.train import Trainer
    spec = CONFIGS["c1"]
    params = []
    for graph in (False, True):
        m, cfg = build("c1", 0.0)
        big, small = batches(cfg, spec, 1)[0], batches(cfg, spec, 1, batch=2)[0]
        tr = Trainer(m, lr=1e-3, graph=graph)
        for i in range(8):
            tr.step(*(big if i % 2 == 0 else small))
        if graph:
            assert len(tr._caps) == 2
        params.append(tr.store.flat.clone())
    assert torch.equal(params[0], params[1])


def test_graphed_forward_sees_weight_updates():
    """asrx.infer.GraphedForward after the weights change (in-place update, as optimizer.step() does): the replay
    re-casts the bf16 operand copy and equals a fresh eager forward; re-binding the parameters (load_state_dict
    into new tensors is the same) makes it capture again."""
    from asrx.infer import GraphedForward
    m, cfg = build("c1", 0.0)
    m.eval()
    s, t, k = batches(cfg, CONFIGS["c1"], 1)[0]
    fwd = GraphedForward(m)
    with torch.no_grad():
        out0 = fwd(s, t[:, :-1], k[:, :-1]).clone()
        for p in m.parameters():
            p.mul_(1.05)
        out1 = fwd(s, t[:, :-1], k[:, :-1]).clone()
        ref1 = m(s, t[:, :-1], k[:, :-1])
    assert not torch.equal(out0, out1)
    assert torch.equal(out1, ref1)
    with torch.no_grad():
        for p in m.parameters():
            p.data = p.data * 0.5          # new storage: the flat store is rebuilt, the old graph dropped
        out2 = fwd(s, t[:, :-1], k[:, :-1]).clone()
        ref2 = m(s, t[:, :-1], k[:, :-1])
    assert torch.equal(out2, ref2)


def test_graph_pool_block_reuse_breaks_write_once_buffers():
    """Cause of the round-5 graph fault: the reverted experiment allocated the grouped
    weight-gradient table DURING the capture and wrote it once, outside the replayed work.  Torch's graph pool hands
    a block freed earlier in the same capture to a later allocation of the capture, so on every replay the kernels
    of the block's earlier tenant write into the "write-once" table before its reader runs — the first replay read
    garbage group pointers (hipErrorIllegalAddress).  Per-replay uploads are immune (the upload is a captured launch
    right before its reader, in stream order), and the shipped device-resident tile / block maps are allocated only
    outside a capture (asrx.kernels._grouped_xcd).  This test reproduces the aliasing without a fault."""
    n = 1 << 16
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x = torch.empty(n, dtype=torch.int32, device=dev)
        x.fill_(1)                     # the earlier tenant's captured kernel
        px = x.data_ptr()
        del x
        table = torch.empty(n, dtype=torch.int32, device=dev)   # the pool reuses x's block
        out = table + 0                # the table's captured reader
    assert table.data_ptr() == px
    table.fill_(7)                     # "written once", outside the graph
    g.replay()
    torch.cuda.synchronize()
    assert bool((out == 1).all()), "the replay's earlier kernel overwrote the write-once buffer"
    assert bool((table == 1).all())


def test_grouped_const_maps_allocated_outside_capture():
    """The shipped form of write-once graph data: the grouped launch's shape-only maps (asrx.kernels._CONST_MAPS)
    are created only when no capture is underway, so they never come from a graph's private pool; a plan first met
    inside a capture takes the per-call buffer with a captured upload instead."""
    from asrx import kernels as K
    from asrx.train import Trainer
    m, cfg = build("c1", 0.0)
    data = batches(cfg, CONFIGS["c1"], 4)
    # (never cleared here: graphs captured earlier in the process point at these buffers)
    tr = Trainer(m, lr=1e-3, graph=True)
    for b in data:                     # eager warm-up steps, then the capture and replays
        tr.step(*b)
    torch.cuda.synchronize()
    assert tr._cap is not None
    assert K._CONST_MAPS, "no device-resident map was created outside the capture"
    for cdev, _, _ in K._CONST_MAPS.values():
        assert cdev.is_cuda and cdev.numel() > 0
