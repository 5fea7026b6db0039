"""Data-parallel backward on the GPU with 2 ranks sharing cuda:0 over gloo: the gradient ranges released
during the backward (decoder, upper encoder half) plus finish() give exactly world x the single-rank
gradients (identical shards), i.e. the overlapped all-reduce neither misses nor double-counts a range and the
split weight-gradient flushes do not change any value."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["ASRX_DP_RELEASE_LAYERS"] = "1"   # fixed one-layer groups (the default, by tile rounds, keeps c1's
    #                                              small encoder whole): the mid-encoder release path
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import asrx
    from asrx.functions import make_ctx, model_backward, model_forward
    from asrx import kernels as K
    from asrx.dist import GradAllReduce
    from oracle.ref_model import CONFIGS, det_params, synthetic_batch
    spec = CONFIGS["c1"]
    cfg = spec["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                         cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    m = m.cuda().train()
    s, t, mk = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=5)
    s, t, mk = s.cuda(), t.cuda(), mk.cuda()

    def grads(ready):
        C = make_ctx(m, 0.0)
        logits, S = model_forward(C, m, s, t[:, :-1], mk[:, :-1])
        _, dl, _ = K.cross_entropy(logits, m.decoder._classifier.V, t[:, 1:].reshape(-1).contiguous())
        C.store.grad.zero_()
        model_backward(C, m, S, dl.to(C.cd), ready=ready)
        return C.store

    st = grads(None)
    ref = st.grad.clone()
    spans = []
    grads(lambda a, b: spans.append((a, b)))       # released-range flushing alone must not change any value
    torch.cuda.synchronize()
    split_ok = bool(torch.equal(st.grad, ref))
    bad0 = (st.grad != ref).nonzero().flatten()
    split_info = (int(bad0.min()), int(bad0.max()), int(bad0.numel())) if bad0.numel() else None
    red = GradAllReduce(st.grad, bucket_mb=1)

    def ready(a, b):        # gloo stages CUDA tensors through the host without waiting on torch's stream (RCCL
        torch.cuda.synchronize()   # orders itself after the queued compute); the test syncs for it
        red.ready(a, b)
    grads(ready)
    torch.cuda.synchronize()
    n_ready = len(red._issued)
    red_ranges = list(red._issued)
    red.finish()
    torch.cuda.synchronize()
    bad = (st.grad != ref * world).nonzero().flatten()
    info = (int(bad.min()), int(bad.max()), int(bad.numel()), red_ranges, st.grad.numel()) if bad.numel() else None
    q.put((rank, n_ready, bool(torch.equal(st.grad, ref * world)),
           (float((st.grad - ref * world).abs().max()), info, split_ok, split_info, spans)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_overlapped_allreduce_exact():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, n_ready, exact, err in res:
        assert n_ready >= 2, n_ready          # decoder + upper encoder half (+ _norm_out) released early
        assert exact, err


def _rehearsal_worker(port, wire, cname, early, q):
    """One-rank RCCL group with the gradient exchange forced on (asrx.dist.FORCE): the multi-GPU step path of a
    graph-mode Trainer — backward captured in segments, RCCL all-reduce (or the bf16 wire's all-to-all + chunk sum
    + all-gather) between the segment replays — against the plain single-GPU Trainer from the same weights."""
    import copy
    import torch.distributed as dist
    os.environ["ASRX_DP_FORCE"] = "1"
    os.environ["ASRX_DP_EARLY_ADAM"] = str(early)   # optional: AdamW of released ranges on a side stream
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    torch.cuda.set_device(0)
    import asrx
    from asrx import dist as D
    from asrx.train import GRAPH_WARMUP, Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch
    spec = CONFIGS[cname]
    cfg = spec["cfg"]
    batch = spec["batch"] if cname == "c1" else 2    # c3 dims (its release groups close: 5 + 5 layers) at B = 2
    torch.manual_seed(0)
    m0 = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                          cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    m1 = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                          cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    m1.load_state_dict(copy.deepcopy(m0.state_dict()))
    s, t, mk = synthetic_batch(cfg, batch, spec["frames"], spec["text_len"] + 1, seed=7)
    s, t, mk = s.cuda(), t.cuda(), mk.cuda()
    out = {}
    for name, m, force in (("dp", m0, True), ("ref", m1, False)):
        D.FORCE = force
        tr = Trainer(m.cuda().train(), lr=1e-3, graph=True, wire=wire, bucket_mb=1)
        losses = [float(tr.step(s, t, mk)) for _ in range(GRAPH_WARMUP + 3)]
        torch.cuda.synchronize()
        out[name] = (tr.store.flat.detach().clone().cpu(), losses, tr.reducer.active, tr._cap is not None)
    (p_dp, l_dp, act_dp, g_dp), (p_ref, l_ref, act_ref, g_ref) = out["dp"], out["ref"]
    err = float((p_dp - p_ref).abs().max() / p_ref.abs().max())
    q.put((act_dp, act_ref, g_dp, g_ref, bool(torch.equal(p_dp, p_ref)), err, l_dp, l_ref))
    dist.destroy_process_group()


@pytest.mark.parametrize("wire,cname,early", [("fp32", "c1", 0), ("bf16", "c1", 0), ("fp32", "c3", 0),
                                              ("fp32", "c3", 1)])
def test_rccl_one_rank_rehearsal_matches_single_gpu(wire, cname, early):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rehearsal_worker, args=(_free_port(), wire, cname, early, q))
    p.start()
    act_dp, act_ref, g_dp, g_ref, exact, err, l_dp, l_ref = q.get(timeout=600)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert act_dp and not act_ref and g_dp and g_ref
    if wire == "fp32":   # a one-rank fp32 all-reduce is the identity: bit-identical training
        assert exact, (err, l_dp, l_ref)
    else:                # one bf16 rounding of every gradient per step
        assert err < 2e-2, (err, l_dp, l_ref)
