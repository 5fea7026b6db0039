"""Headline benchmark: encoder+decoder frames/s of the c3 training step (BASELINE.json configs[2]:
12+12 layers, d_model 512, h 8, ff 2048, batch 64 per GPU, T=1000 frames of 80-bin log-mel, L=64 tokens,
bf16, dropout 0.1, fused AdamW), data-parallel over N GPUs (weak scaling: 64 utterances per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Prints ONE JSON line (rank 0). `value` = all ranks' frames / max-over-ranks wall time of the K timed steps.
`roofline` = the dominant GEMM kernel instantiation (largest total time in the last warmup step, named as
rocprofv3 names it), timed live with HIP events on its launch stream over the timed steps; `sub_rooflines` = the
north_star's per-kernel figures (attention projection GEMM and fused attention: MFMA fraction; LayerNorm and the
unfused softmax: HBM fraction) at the workload's encoder shapes, after the timed region; `cpu_baseline` = the
oracle (fp32 eager PyTorch restatement of the reference) train step on the host cores, bounded sample, rank 0 at
N=1 only.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="skip the per-kernel sub-rooflines")
    return ap.parse_args()


def cpu_baseline(cfg, frames, text_len, batch, steps):
    """Oracle train step (fp32 eager CPU restatement of the reference, per-head loop) on the host cores."""
    from oracle.ref_model import det_params, synthetic_batch, train_step_grads
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    P = {k: v.clone().requires_grad_(True) for k, v in det_params(cfg, 0).items()}
    s, t, m = synthetic_batch(cfg, batch, frames, text_len + 1, seed=99)
    train_step_grads(P, s, t, m, cfg, training=True)          # warmup
    t0 = time.perf_counter()
    for _ in range(steps):
        for v in P.values():
            v.grad = None
        train_step_grads(P, s, t, m, cfg, training=True)
    dt = time.perf_counter() - t0
    return {"value": round(batch * frames * steps / dt, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle fp32 train step (fwd+CE+bwd, dropout {cfg.dropout}) {cfg.n_enc}+{cfg.n_dec} layers "
                      f"d{cfg.d_model}, B={batch}, T={frames}, L={text_len}, {steps} steps after 1 warmup, "
                      f"{dt:.1f}s"}


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the committed PMC summary (profiles/*pmc*.json, written by
    tools/pmc_table.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), or None."""
    path = os.path.join(REPO, "profiles", f"{config}_pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if rec is None else rec["hbm_bytes_per_launch"]


def _graph_time_ms(fn, launches=20, rounds=5):
    """GPU time of one fn() call: `launches` calls captured in a HIP graph, replayed between HIP events on the
    capturing stream (no host launch gaps inside the timed region); median over rounds."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(launches):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / launches)
    return sorted(ts)[len(ts) // 2]


def sub_rooflines(B, T2, d, H, ff, p_drop):
    """The north_star's per-kernel sub-rooflines at the workload's encoder shapes (rows = B*T'): MFMA
    utilisation of the attention projection GEMM and the fused attention forward, HBM fraction of LayerNorm
    fwd/bwd and of the (unfused-path) masked softmax.  Algorithmic bytes: every operand read once, every
    output written once."""
    from asrx import kernels as K
    from asrx.kernels import MaskSpec
    rows, dh = B * T2, d // H
    gen = torch.Generator(device="cuda").manual_seed(7)
    out = {}

    def mfma(name, flops, fn, note):
        t = _graph_time_ms(fn)
        tf = flops / (t * 1e-3) / 1e12
        out[name] = {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / PEAK_BF16_TFLOPS, 4), "us": round(t * 1e3, 2), "shape": note}

    def hbm(name, nbytes, fn, note):
        t = _graph_time_ms(fn)
        gbs = nbytes / (t * 1e-3) / 1e9
        out[name] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(gbs / PEAK_HBM_GBS, 4), "us": round(t * 1e3, 2), "shape": note}

    x = (torch.randn(rows, d, device="cuda", generator=gen) * 0.5).bfloat16()
    wqkv = (torch.randn(3 * d, d, device="cuda", generator=gen) * 0.05).bfloat16()
    bqkv = torch.randn(3 * d, device="cuda", generator=gen) * 0.1
    qkv = torch.empty(rows, 3 * d, device="cuda", dtype=torch.bfloat16)
    mfma("qkv_projection_gemm", 2.0 * rows * 3 * d * d, lambda: K.linear(x, wqkv, qkv, bias=bqkv),
         f"[{rows}x{d}] x [{d}x{3 * d}] + bias, bf16 out")
    o = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    st = ((3 * d, T2 * 3 * d),) * 3 + ((d, T2 * d),)
    dm = K.dropmask_buffer(B, H, T2, T2, dh, p_drop, x.device)
    mfma("attention_fwd", 4.0 * B * H * T2 * T2 * dh,
         lambda: K.attention_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], o, B, H, T2, T2, dh, st, d ** -0.5,
                                 MaskSpec(), p_drop, 11, dropmask=dm),
         f"B*H={B * H} Lq=Lk={T2} dh={dh}, dropout {p_drop} (incl. the keep-bit generation kernel)")
    xr = torch.randn(rows, d, device="cuda", generator=gen)
    gam = torch.rand(d, device="cuda", generator=gen) + 0.5
    bet = torch.randn(d, device="cuda", generator=gen)
    y = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    mean, rstd = K.layernorm_fwd(xr, gam, bet, y)
    hbm("layernorm_fwd", rows * d * (4 + 2) + rows * 8, lambda: K.layernorm_fwd(xr, gam, bet, y),
        f"[{rows}x{d}] fp32 in, bf16 out, fp32 mean/rstd")
    dy = torch.randn(rows, d, device="cuda", generator=gen).bfloat16()
    dres = torch.randn(rows, d, device="cuda", generator=gen)
    dxd = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    dgb = torch.zeros(2 * d, device="cuda")
    hbm("layernorm_bwd", rows * d * (4 + 2 + 4 + 4 + 2) + rows * 8,
        lambda: K.layernorm_bwd(xr, dy, gam, mean, rstd, dgb, dres=dres, dx_drop=dxd, dropout_p=p_drop, seed=5,
                                defer=[]),
        f"[{rows}x{d}]: x fp32, dy bf16, dres fp32 in; dx fp32, dropout(dx) bf16 out")
    nbh, ld = B * H, (T2 + 7) // 8 * 8
    sc = torch.randn(nbh, T2, ld, device="cuda", generator=gen).bfloat16()
    pr = torch.empty_like(sc)
    hbm("softmax_fwd", 2 * nbh * T2 * T2 * 2, lambda: K.softmax_fwd(sc, pr, None, nbh, H, T2, T2, ld, d ** -0.5,
                                                                    MaskSpec()),
        f"unfused path (attention=\"unfused\"): {nbh}x{T2}x{T2} bf16 scores -> probabilities")
    dpd = torch.randn(nbh, T2, ld, device="cuda", generator=gen).bfloat16()
    dsc = torch.empty_like(sc)
    hbm("softmax_bwd", 3 * nbh * T2 * T2 * 2, lambda: K.softmax_bwd(pr, dpd, dsc, nbh, T2, T2, ld, d ** -0.5),
        f"unfused path: {nbh}x{T2}x{T2} bf16 probabilities + their gradient -> score gradient")
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import asrx
    from asrx import kernels as K
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch

    spec = CONFIGS[args.config]
    cfg = spec["cfg"]
    B = args.batch or spec["batch"]
    T, L = spec["frames"], spec["text_len"]
    torch.manual_seed(0)
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    if world > 1:   # identical initial weights on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    trainer = Trainer(model, lr=1e-4)
    s, t, m = synthetic_batch(cfg, B, T, L + 1, seed=1234 + rank)
    s, t, m = s.cuda(), t.cuda(), m.cuda()

    for i in range(args.warmup):
        survey = not args.no_probe and i == args.warmup - 1
        if survey:      # last warmup step: time every GEMM launch to find the dominant kernel instantiation
            K.PROBE = K.KernelProbe()
            K.PROBE.active = True
        loss = trainer.step(s, t, m)
    torch.cuda.synchronize()
    probe = None
    if K.PROBE is not None:
        probe = K.KernelProbe(K.PROBE.dominant())
        probe.active = True
        K.PROBE = probe
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(s, t, m)
    t_enq = time.perf_counter() - t0      # host time to enqueue the K steps (the GPU runs behind it)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    K.PROBE = None
    if world > 1:
        x = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        dt = float(x)
    frames = B * T * args.steps * world
    value = frames / dt
    roof = None
    if probe is not None and probe.events.get(probe.target):
        durs = probe.durations_ms(probe.target)
        avg_ms = sum(durs) / len(durs)
        achieved = probe.flops[probe.target] / (sum(durs) * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": pmc_traffic(probe.target, args.config),
                "kernel": probe.target, "launches_per_step": len(durs) // args.steps,
                "avg_launch_us": round(avg_ms * 1e3, 2),
                "flop_per_launch_avg": probe.flops[probe.target] // len(durs)}
    out = {"metric": "encoder+decoder frames/sec/GPU at d_model=512 T=1000; 1->8 GPU scaling",
           "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random-init weights)",
           "config": {"workload": f"{args.config}: {cfg.n_enc}+{cfg.n_dec} layers d_model={cfg.d_model} "
                                  f"h={cfg.n_heads} ff={cfg.ff_dim}, B={B}/GPU, T={T} (T'={asrx.subsampled(T)}), "
                                  f"L={L}, V={cfg.vocab_size}; bf16 train step fwd+CE+bwd+AdamW, dropout "
                                  f"{cfg.dropout}",
                      "model": "speech-transformer", "global_batch": B * world, "seq_len": T,
                      "parallelism": f"dp{world}"},
           "frames_per_sec_per_gpu": round(value / world, 1),
           "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
           "loss": round(float(loss), 4),
           "roofline": roof}
    if rank == 0 and not args.no_sub:
        out["sub_rooflines"] = sub_rooflines(B, asrx.subsampled(T), cfg.d_model, cfg.n_heads, cfg.ff_dim,
                                             cfg.dropout)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, T, L, args.cpu_batch, args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
