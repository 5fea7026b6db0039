"""Data-parallel gradient exchange on CPU: world_size 2 over gloo, and an injected fake all-reduce.

The product uses RCCL (backend "nccl") on the GPUs; the bucketing / ordering / averaging logic is
backend-independent and is exercised here with gloo."""
import os
import socket

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.ref_model import CONFIGS, det_params, synthetic_batch, train_step_grads


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flatten(grads, keys):
    return torch.cat([grads[k].reshape(-1) if grads[k] is not None else torch.zeros(0) for k in keys])


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from asrx.dist import GradAllReduce
    spec = CONFIGS["micro"]
    cfg = spec["cfg"]
    s, t, m = synthetic_batch(cfg, 4, spec["frames"], spec["text_len"] + 1, seed=11)
    # equal-length shards so that the mean of per-shard mean losses equals the full-batch mean loss
    t[:, -1] = 7
    m[:] = 1.0
    sh = slice(rank * 2, rank * 2 + 2)
    P = {k: v.clone().requires_grad_(True) for k, v in det_params(cfg).items()}
    _, grads = train_step_grads(P, s[sh], t[sh], m[sh], cfg, training=False)
    keys = sorted(k for k in grads if grads[k] is not None)
    flat = _flatten(grads, keys)
    red = GradAllReduce(flat, bucket_mb=0.05)   # many small buckets
    assert len(red.buckets) > 3
    red()
    flat /= red.world
    q.put((rank, flat))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_ws2_allreduce_equals_full_batch():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = CONFIGS["micro"]
    cfg = spec["cfg"]
    s, t, m = synthetic_batch(cfg, 4, spec["frames"], spec["text_len"] + 1, seed=11)
    t[:, -1] = 7
    m[:] = 1.0
    P = {k: v.clone().requires_grad_(True) for k, v in det_params(cfg).items()}
    _, grads = train_step_grads(P, s, t, m, cfg, training=False)
    keys = sorted(k for k in grads if grads[k] is not None)
    full = _flatten(grads, keys)
    assert torch.allclose(res[0], res[1])
    assert float((res[0] - full).abs().max() / full.abs().max()) < 1e-5


def test_bucketing_fake_backend_order_and_coverage():
    from asrx.dist import GradAllReduce, bucket_views
    flat = torch.arange(1000, dtype=torch.float32)
    seen = []

    def fake(b):
        seen.append((b.data_ptr(), b.numel()))
        b.mul_(3.0)             # a "world of 3" replicas holding identical grads
    fake.world = 3
    r = GradAllReduce(flat, bucket_mb=256 * 4 / 2 ** 20, allreduce_fn=fake)
    assert [v.numel() for v in r.buckets] == [256, 256, 256, 232]
    r()
    # issued in reverse bucket order, every element exactly once
    assert [n for _, n in seen] == [232, 256, 256, 256]
    assert seen[0][0] > seen[-1][0]
    assert torch.equal(flat, torch.arange(1000, dtype=torch.float32) * 3)
    assert r.world == 3
    assert sum(v.numel() for v in bucket_views(torch.zeros(10), 3)) == 10


def test_ready_ranges_overlap_then_finish_covers_complement():
    """Ranges released during the backward are reduced once each; finish() reduces exactly the rest."""
    from asrx.dist import GradAllReduce
    flat = torch.ones(1000)
    counts = torch.zeros(1000)
    base = flat.data_ptr()

    def fake(b):
        o = (b.data_ptr() - base) // 4
        counts[o:o + b.numel()] += 1
        b.mul_(2.0)
    fake.world = 2
    r = GradAllReduce(flat, bucket_mb=100 * 4 / 2 ** 20, allreduce_fn=fake)
    r.ready(700, 1000)          # decoder span
    r.ready(400, 700)           # upper encoder half
    assert counts[400:].eq(1).all() and counts[:400].eq(0).all()
    r.finish()
    assert counts.eq(1).all() and flat.eq(2.0).all()
    r.ready(0, 10)              # the next step starts from a clean slate
    r.finish()
    assert counts.eq(2).all()


def _ready_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from asrx.dist import GradAllReduce
    flat = torch.arange(5000, dtype=torch.float32) * (rank + 1)
    r = GradAllReduce(flat, bucket_mb=0.002)
    r.ready(3000, 5000)
    r.ready(1234, 3000)
    r.finish()
    q.put((rank, flat))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_ws2_ready_ranges():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ready_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.arange(5000, dtype=torch.float32) * 3
    assert torch.equal(res[0], want) and torch.equal(res[1], want)


def _torch_chunk_sum(recv, W, c, out):
    """Test double of asrx_sum_chunks_bf16 (CPU tensors): fp32 sum of the W bf16 copies, one rounding."""
    out.copy_(recv.view(W, c).float().sum(0).to(torch.bfloat16))


def _bf16_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from asrx.dist import GradAllReduce
    g = torch.Generator().manual_seed(100 + rank)
    flat = torch.randn(5003, generator=g)
    r = GradAllReduce(flat, bucket_mb=0.004, wire="bf16", chunk_sum=_torch_chunk_sum)   # ragged buckets
    assert len(r.buckets) > 3
    r.ready(2000, 5003)
    r.finish()
    q.put((rank, flat))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_ws3_bf16_wire_fp32_sum():
    """bf16 wire: every rank ends with bf16(sum_r bf16(g_r)) — the sum in fp32, one rounding of each rank's
    gradient and one of the sum — identical on all ranks; world 3 (chunks do not divide the buckets)."""
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bf16_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = [torch.randn(5003, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)]
    want = sum(p.to(torch.bfloat16).float() for p in parts).to(torch.bfloat16).float()
    exact = sum(parts)
    for r in range(world):
        assert torch.equal(res[r], want)
    assert float((res[0] - exact).abs().max() / exact.abs().max()) < 2 ** -7


def test_release_groups_cover_each_parameter_once():
    """The multi-GPU backward's release schedule (functions.release_groups + _spans over the flat store) followed
    by the reducer's finish() reduces every gradient element exactly once, for every release granularity."""
    import asrx
    from asrx.dist import GradAllReduce
    from asrx.functions import _spans, param_order, release_groups
    from asrx.params import FlatParams
    cfg = CONFIGS["c2"]["cfg"]
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    store = FlatParams(param_order(model), torch.device("cpu"))   # the product's flat layout (built on the host)

    class _C:
        pass
    C = _C()
    C.store = store
    enc, n = model.encoder, len(model.encoder._layers)
    for every in (0, 1, 2, 4, 5, n, n + 3):
        flat = store.grad
        counts = torch.zeros(flat.numel())
        base = flat.data_ptr()

        def fake(b):
            o = (b.data_ptr() - base) // 4
            counts[o:o + b.numel()] += 1
        fake.world = 2
        r = GradAllReduce(flat, bucket_mb=0.25, allreduce_fn=fake)
        released = list(model.decoder.parameters())
        for a, b in _spans(C, released):
            r.ready(a, b)
        groups = release_groups(n, every)
        assert groups == sorted(groups, reverse=True) and all(lo > 0 for lo, _ in groups)
        for lo, hi in groups:
            ps = [p for l in enc._layers[lo:hi] for p in l.parameters()]
            if hi == n:
                ps += list(enc._norm_out.parameters())
            for a, b in _spans(C, ps):
                r.ready(a, b)
        r.finish()
        assert counts.eq(1).all(), every


def test_bench_gpus_flag_launches_ranks_on_cpu():
    """`python bench.py --gpus 2` with no launcher environment starts the two ranks itself (child
    torch.distributed.run, gloo self-test mode: no GPU) and relays rank 0's single JSON line with n_gpus = 2;
    a rank whose WORLD_SIZE disagrees with --gpus exits non-zero."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    bench = os.path.join(REPO, "bench.py")
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--steps", "3", "--warmup", "0", "--cpu-dist-selftest"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3
    env_bad = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--cpu-dist-selftest"], env=env_bad,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0


def _release_worker(rank, world, port, q):
    """One rank of the multi-GPU backward's release schedule over the product's flat gradient layout (c2 model):
    decoder spans first, then each encoder release group, then finish() — as asrx.functions.encoder_bwd issues
    them — with gradients that differ per rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    import asrx
    from asrx.dist import GradAllReduce
    from asrx.functions import _spans, param_order, release_groups
    from asrx.params import FlatParams
    cfg = CONFIGS["c2"]["cfg"]
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16")
    store = FlatParams(param_order(model), torch.device("cpu"))

    class _C:
        pass
    C = _C()
    C.store = store
    enc, n = model.encoder, len(model.encoder._layers)
    out = {}
    for every in (0, 1, 4, n):
        flat = store.grad
        flat.copy_(torch.arange(flat.numel(), dtype=torch.float32).remainder_(977.0) * (rank + 1) + rank)
        # 0.37 MB buckets: ragged against every span, so each rank count cuts the released ranges differently
        r = GradAllReduce(flat, bucket_mb=0.37)
        for a, b in _spans(C, list(model.decoder.parameters())):
            r.ready(a, b)
        for lo, hi in release_groups(n, every):
            ps = [p for l in enc._layers[lo:hi] for p in l.parameters()]
            if hi == n:
                ps += list(enc._norm_out.parameters())
            for a, b in _spans(C, ps):
                r.ready(a, b)
        r.finish()
        base = torch.arange(flat.numel(), dtype=torch.float32).remainder_(977.0)
        want = base * sum(w + 1 for w in range(world)) + sum(range(world))
        out[every] = (bool(torch.equal(flat, want)), float(flat.double().sum()))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_ws4_release_schedule_sums_every_element_once():
    """World size 4 (beyond the 2- and 3-rank cases): the released ranges plus finish() leave every rank holding
    the exact sum over ranks of every gradient element, for the default and fixed release granularities."""
    world, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_release_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for every in res[0]:
        for r in range(world):
            assert res[r][every][0], (r, every)                  # exact sum over ranks, every element once
            assert res[r][every][1] == res[0][every][1], (r, every)
