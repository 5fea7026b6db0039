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
import subprocess
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
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-steps", type=int, default=4)
    ap.add_argument("--no-graph", action="store_true", help="eager steps (no HIP graph capture)")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="skip the per-kernel sub-rooflines")
    ap.add_argument("--no-other", action="store_true", help="skip the c2 / c5 forward configs")
    ap.add_argument("--cpu-dist-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def host_cpu():
    """(model name, logical CPUs in this process's affinity set, threads to use).  The threads are the CPU share
    the box grants this job (OMP_NUM_THREADS, 16 per GPU on the pool), at most the affinity set."""
    model = "unknown"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS") or aff)
    return model, aff, max(1, min(aff, share))


def cpu_baseline(cfg, frames, text_len, batch, steps, extra=True):
    """The reference's CPU PyTorch path on the host cores: the oracle (fp32 eager restatement of the
    reference, per-head loop, nan_to_num) timed on a bounded sample of the headline workload — the c3 train
    step at B=8 — plus, with `extra`, the forward of every GPU config (c2 at full batch, c3 at
    B=64, c5 at B=2) normalised to frames/s."""
    from oracle.ref_model import CONFIGS, det_params, forward, synthetic_batch, train_step_grads
    model, aff, threads = host_cpu()
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
    out = {"value": round(batch * frames * steps / dt, 1), "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": f"oracle fp32 train step (fwd+CE+bwd, dropout {cfg.dropout}) {cfg.n_enc}+{cfg.n_dec} layers "
                     f"d{cfg.d_model}, B={batch}, T={frames}, L={text_len}, {steps} steps after 1 warmup, "
                     f"{dt:.1f}s",
           "cpu_model": model, "affinity_cpus": aff, "threads": threads,
           "frames_per_s_per_thread": round(batch * frames * steps / dt / threads, 1),
           # the GPU pool grants each GPU a share of the host (OMP_NUM_THREADS, 16 per GPU) and asks worker pools to
           # stay within it; the affinity set is the whole shared machine, so the baseline runs at the share
           "threads_rule": "OMP_NUM_THREADS share of the box (the pool's per-GPU CPU share), not the affinity set"}
    if extra:
        fw = {}
        for name, b in (("c2", CONFIGS["c2"]["batch"]), ("c3", 64), ("c5", 2)):
            sp = CONFIGS[name]
            c = sp["cfg"]
            Pn = det_params(c, 0)
            sx, tx, mx = synthetic_batch(c, b, sp["frames"], sp["text_len"] + 1, seed=99)
            with torch.no_grad():
                t0 = time.perf_counter()
                forward(Pn, sx, tx[:, :-1], mx[:, :-1], c, False)
                d1 = time.perf_counter() - t0
            fw[name] = {"frames_per_s": round(b * sp["frames"] / d1, 1), "batch": b, "frames": sp["frames"],
                        "s": round(d1, 2), "mode": "fp32 forward (eval)"}
        out["forward"] = fw
    return out


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


def pmc_mfma(kernel, config):
    """MFMA busy fraction of `kernel` from the committed counter pass (profiles/<config>_pmc_mfma.json, written by
    tools/pmc_mfma.py from rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE),
    or None."""
    path = os.path.join(REPO, "profiles", f"{config}_pmc_mfma.json")
    try:
        with open(path) as f:
            rec = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    if rec is None:
        return None
    return {k: rec.get(k) for k in ("mfma_busy_frac", "mfma_tflops", "clock_ghz", "mfma_flop_per_launch")}


def _graph_time_ms(fns, launches=24, rounds=5):
    """GPU time of one launch: `launches` calls (cycling through the closures `fns`) captured in a HIP graph,
    replayed between HIP events on the capturing stream (no host launch gaps inside the timed region); median
    over rounds."""
    for fn in fns:
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(launches):
            fns[i % len(fns)]()
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


COLD_BYTES = 768 << 20    # > the 256 MiB Infinity Cache: rotating buffer sets this large read from HBM


def sub_rooflines(B, T2, d, H, ff, p_drop):
    """The north_star's per-kernel sub-rooflines at the workload's encoder shapes (rows = B*T'): MFMA
    utilisation of the attention projection GEMM and the fused attention forward, HBM fraction of LayerNorm
    fwd/bwd and of the (unfused-path) masked softmax.  Algorithmic bytes: every operand read once, every
    output written once.

    Cache state: `us` / `frac` rotate through independent buffer sets totalling > 768 MiB, so every launch
    reads operands the previous launches evicted from the 256 MiB Infinity Cache (cold, HBM-sourced);
    `us_warm` / `frac_warm` repeat one buffer set (its working set stays cache-resident)."""
    from asrx import kernels as K
    from asrx.kernels import MaskSpec
    rows, dh = B * T2, d // H
    gen = torch.Generator(device="cuda").manual_seed(7)
    out = {}

    def timed(make, set_bytes):
        nsets = max(2, -(-COLD_BYTES // set_bytes))
        fns = [make() for _ in range(nsets)]
        t_cold = _graph_time_ms(fns)
        t_warm = _graph_time_ms(fns[:1])
        del fns
        torch.cuda.empty_cache()
        return t_cold, t_warm, nsets

    def mfma(name, flops, make, set_bytes, note):
        t, tw, n = timed(make, set_bytes)
        tf, tfw = flops / (t * 1e-3) / 1e12, flops / (tw * 1e-3) / 1e12
        out[name] = {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / PEAK_BF16_TFLOPS, 4), "us": round(t * 1e3, 2),
                     "frac_warm": round(tfw / PEAK_BF16_TFLOPS, 4), "us_warm": round(tw * 1e3, 2),
                     "buffer_sets": n, "shape": note}

    def make_copy(nbytes):
        # the same byte count as a plain device copy (half read, half written; torch's vectorised copy kernel, fp32
        # elements in 16-B vectors): what one launch of this size reaches on this box from HBM — the floor the
        # kernel's cold fraction is to be read against (a reference point, not product code)
        src = torch.empty(max(1, nbytes // 8), device="cuda")
        dst = torch.empty_like(src)
        return lambda: dst.copy_(src)

    def hbm(name, nbytes, make, note):
        t, tw, n = timed(make, nbytes)
        gbs, gbw = nbytes / (t * 1e-3) / 1e9, nbytes / (tw * 1e-3) / 1e9
        tc, _, _ = timed(lambda: make_copy(nbytes), nbytes)
        gbc = nbytes / (tc * 1e-3) / 1e9
        out[name] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(gbs / PEAK_HBM_GBS, 4), "us": round(t * 1e3, 2),
                     "frac_warm": round(gbw / PEAK_HBM_GBS, 4), "us_warm": round(tw * 1e3, 2),
                     "buffer_sets": n, "shape": note,
                     "copy_floor": {"frac": round(gbc / PEAK_HBM_GBS, 4), "us": round(tc * 1e3, 2),
                                    "kernel_vs_copy": round(tc / t, 3)}}

    def rnd(*shape, dtype=torch.float32, scale=1.0):
        return (torch.randn(*shape, device="cuda", generator=gen) * scale).to(dtype)

    wqkv = rnd(3 * d, d, dtype=torch.bfloat16, scale=0.05)
    bqkv = rnd(3 * d, scale=0.1)

    def make_qkv():
        x, qkv = rnd(rows, d, dtype=torch.bfloat16, scale=0.5), torch.empty(rows, 3 * d, device="cuda",
                                                                              dtype=torch.bfloat16)
        return lambda: K.linear(x, wqkv, qkv, bias=bqkv)
    mfma("qkv_projection_gemm", 2.0 * rows * 3 * d * d, make_qkv, rows * d * 8,
         f"[{rows}x{d}] x [{d}x{3 * d}] + bias, bf16 out")
    st = ((3 * d, T2 * 3 * d),) * 3 + ((d, T2 * d),)

    def make_attn():
        qkv = rnd(rows, 3 * d, dtype=torch.bfloat16, scale=0.5)
        o = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
        dm = K.dropmask_buffer(B, H, T2, T2, dh, p_drop, qkv.device)
        return lambda: K.attention_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], o, B, H, T2, T2, dh, st, d ** -0.5,
                                       MaskSpec(), p_drop, 11, dropmask=dm)
    mfma("attention_fwd", 4.0 * B * H * T2 * T2 * dh, make_attn, rows * d * 8,
         f"B*H={B * H} Lq=Lk={T2} dh={dh}, dropout {p_drop} (incl. the keep-bit generation kernel)")
    # its memory side: Q, K, V read once, O written once (bf16), keep bits written and read (1 bit per score, two
    # layouts) — the c3 shape's arithmetic intensity (~100 FLOP/B) is below the MI355X ridge (2.5 PF / 8 TB/s = 312),
    # so an MFMA fraction near 30% is the HBM roof here
    a_bytes = 4 * rows * d * 2 + 3 * B * H * T2 * T2 / 8
    at = out["attention_fwd"]
    at["algorithmic_bytes"] = int(a_bytes)
    at["hbm_frac"] = round(a_bytes / (at["us"] * 1e-6) / 1e9 / PEAK_HBM_GBS, 4)
    at["mfma_roof_at_hbm_peak"] = round(min(1.0, (4.0 * B * H * T2 * T2 * dh / a_bytes) * PEAK_HBM_GBS * 1e9 /
                                            (PEAK_BF16_TFLOPS * 1e12)), 4)
    gam = torch.rand(d, device="cuda", generator=gen) + 0.5
    bet = rnd(d)

    def make_lnf():
        xr, y = rnd(rows, d), torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
        return lambda: K.layernorm_fwd(xr, gam, bet, y)
    hbm("layernorm_fwd", rows * d * (4 + 2) + rows * 8, make_lnf, f"[{rows}x{d}] fp32 in, bf16 out, fp32 mean/rstd")

    def make_lnb():
        xr = rnd(rows, d)
        mean, rstd = K.layernorm_fwd(xr, gam, bet, torch.empty(rows, d, device="cuda", dtype=torch.bfloat16))
        dy, dres = rnd(rows, d, dtype=torch.bfloat16), rnd(rows, d)
        dxd, dgb = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16), torch.zeros(2 * d, device="cuda")
        return lambda: K.layernorm_bwd(xr, dy, gam, mean, rstd, dgb, dres=dres, dx_drop=dxd, dropout_p=p_drop,
                                       seed=5, defer=[])
    hbm("layernorm_bwd", rows * d * (4 + 2 + 4 + 4 + 2) + rows * 8, make_lnb,
        f"[{rows}x{d}]: x fp32, dy bf16, dres fp32 in; dx fp32, dropout(dx) bf16 out")
    nbh, ld = B * H, (T2 + 7) // 8 * 8

    def make_smf():
        sc = rnd(nbh, T2, ld, dtype=torch.bfloat16)
        pr = torch.empty_like(sc)
        return lambda: K.softmax_fwd(sc, pr, None, nbh, H, T2, T2, ld, d ** -0.5, MaskSpec())
    hbm("softmax_fwd", 2 * nbh * T2 * T2 * 2, make_smf,
        f"unfused path (attention=\"unfused\"): {nbh}x{T2}x{T2} bf16 scores -> probabilities")

    def make_smb():
        pr, dpd = rnd(nbh, T2, ld, dtype=torch.bfloat16), rnd(nbh, T2, ld, dtype=torch.bfloat16)
        dsc = torch.empty_like(pr)
        return lambda: K.softmax_bwd(pr, dpd, dsc, nbh, T2, T2, ld, d ** -0.5)
    hbm("softmax_bwd", 3 * nbh * T2 * T2 * 2, make_smb,
        f"unfused path: {nbh}x{T2}x{T2} bf16 probabilities + their gradient -> score gradient")
    return out


# algorithmic FLOP per input frame of the teacher-forced forward (FlopCounterMode over the reference)
FWD_MFLOP_PER_FRAME = {"c2": 4.21, "c5": 36.44}
PEAK_F32_TFLOPS = 157.3   # MI355X fp32 matrix (= vector) peak (MI355X_MICROARCH.md)


def new_train_step(name="new_small", batch=32, reps=20):
    """The `new/` family's training step as new/train.py:17-34 runs it (forward, CrossEntropyLoss on the shifted
    targets, backward, global-norm clip at 1.0 — asrx.new.clip_grad_norm_, one native reduction — and the caller's
    torch AdamW), eager, fp32 (the variant's own precision), dropout 0.1, at `name`'s dims: utterances/s and
    spectrogram frames/s over `reps` steps after 3 warm-up ones (HIP events)."""
    import asrx.new
    from oracle import ref_model_new as N
    c = N.NEW_CONFIGS[name]
    torch.manual_seed(0)
    m = asrx.new.Transformer(c.vocab_size, c.n_mels, c.enc_seq_len, c.dec_seq_len, c.hidden_dim, c.n_enc, c.n_dec,
                             c.n_heads, c.ff_dim, "cuda", dropout=0.1, sr=c.sr, n_fft=c.n_fft, padding_idx=c.pad_id,
                             eos_token=c.eos_id, bos_token=c.bos_id).cuda().train()
    spectre, lens, text = N.synthetic_batch(c, batch, seed=99)
    true = torch.full_like(text, c.eos_id)
    true[:, :-1] = text[:, 1:]
    b = {"spectre": spectre.cuda(), "spectrogram_len": lens.cuda(), "encoded_text": text.cuda(),
         "text_len": lens.cuda(), "true_text": true.cuda()}
    params = list(m.parameters())
    opt = torch.optim.AdamW(params, lr=1e-4)
    ce = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad()
        loss = ce(m(b).transpose(1, 2), b["true_text"])
        loss.backward()
        asrx.new.clip_grad_norm_(params, 1.0)
        opt.step()
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        loss = step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"metric": "utterances/s (train step: fwd + CE + bwd + clip 1.0 + AdamW, eager)",
            "value": round(batch / (ms * 1e-3), 1), "ms_per_step": round(ms, 3),
            "frames_per_s": round(batch * c.enc_len / (ms * 1e-3), 1), "dtype": "f32", "batch": batch,
            "frames": c.enc_len, "text_len": c.dec_seq_len, "d_model": c.n_mels, "layers": f"{c.n_enc}+{c.n_dec}",
            "loss": round(float(loss.detach()), 4),
            "note": "tiny model (d 80): launch-bound; the variant's own training-script dims (oracle/ref_model_new.py)"}


def other_configs(names=("c2", "c5"), reps=5):
    """The BASELINE.json forward configs beside the headline step, timed after it: c2 (configs[1]: fp32 forward,
    B=32, T=512, 6+6 layers d256) against the fp32 matrix peak and c5 (configs[4]: bf16 forward, B=16, T=4000 ->
    T'=999, the tiled attention path of the long utterances) against the bf16 MFMA peak, as frames/s of the
    teacher-forced forward (model.eval(), no_grad, replayed from a HIP graph by asrx.infer.GraphedForward; HIP
    events around `reps` forwards after 2 warm-up ones; the eager time is reported beside it), plus the
    c5 encoder self-attention forward kernel alone (B*H=128, 999x999, dh=64; graph replay, cold buffers)."""
    import asrx
    from asrx import kernels as K
    from asrx.infer import GraphedForward
    from asrx.kernels import MaskSpec
    from oracle.ref_model import CONFIGS, synthetic_batch
    out = {}
    for name in names:
        spec = CONFIGS[name]
        cfg = spec["cfg"]
        B, T, L = spec["batch"], spec["frames"], spec["text_len"]
        prec = "fp32" if name == "c2" else "bf16"
        torch.manual_seed(0)
        model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                                 cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout,
                                 precision=prec).cuda().eval()
        s, t, m = synthetic_batch(cfg, B, T, L + 1, seed=4321)
        s, t, m = s.cuda(), t[:, :-1].cuda(), m[:, :-1].cuda()
        fwd = GraphedForward(model)           # HIP-graph replay (asrx.infer): no per-launch host cost
        with torch.no_grad():
            for _ in range(2):
                model(s, t, m)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                model(s, t, m)
            e1.record()
            e1.synchronize()
            ms_eager = e0.elapsed_time(e1) / reps
            fwd(s, t, m)
            fwd(s, t, m)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                fwd(s, t, m)
            e1.record()
            e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fps = B * T / (ms * 1e-3)
        tf = FWD_MFLOP_PER_FRAME[name] * 1e6 * B * T / (ms * 1e-3) / 1e12
        peak = PEAK_F32_TFLOPS if prec == "fp32" else PEAK_BF16_TFLOPS
        out[name] = {"metric": "frames/s (teacher-forced forward)", "value": round(fps, 1), "ms_per_forward": round(ms, 3),
                     "dtype": "f32" if prec == "fp32" else "bf16", "batch": B, "frames": T, "text_len": L,
                     "achieved_tflops": round(tf, 1), "peak_tflops": peak, "frac": round(tf / peak, 4),
                     "flop_basis": f"{FWD_MFLOP_PER_FRAME[name]} MFLOP/frame (SURVEY 8(d))",
                     "ms_per_forward_eager": round(ms_eager, 3), "graph": True}
        del model
        torch.cuda.empty_cache()
    if "c5" in names:   # the tiled (Lk > 256) attention forward alone at the c5 encoder shape
        cfg = CONFIGS["c5"]["cfg"]
        B, H, d = CONFIGS["c5"]["batch"], cfg.n_heads, cfg.d_model
        T2, dh = asrx.subsampled(CONFIGS["c5"]["frames"]), d // cfg.n_heads
        gen = torch.Generator(device="cuda").manual_seed(5)
        rows = B * T2
        st = ((3 * d, T2 * 3 * d),) * 3 + ((d, T2 * d),)

        def make():
            qkv = (torch.randn(rows, 3 * d, device="cuda", generator=gen) * 0.5).bfloat16()
            o = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
            return lambda: K.attention_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], o, B, H, T2, T2, dh, st, d ** -0.5,
                                           MaskSpec())
        nsets = max(2, -(-COLD_BYTES // (rows * d * 8)))
        fns = [make() for _ in range(nsets)]
        t_ms = _graph_time_ms(fns)
        flops = 4.0 * B * H * T2 * T2 * dh
        tf = flops / (t_ms * 1e-3) / 1e12
        out["c5"]["attention_fwd"] = {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS,
                                      "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4),
                                      "us": round(t_ms * 1e3, 2),
                                      "shape": f"B*H={B * H} Lq=Lk={T2} dh={dh}, no mask, eval (no dropout)"}
        del fns
        torch.cuda.empty_cache()

        # the training form at the same shape (streamed forward with dropout 0.1 + the O rounding residual, and the
        # key-block backward: 4 blocks of 256 keys per head, dQ shares added in fp32)
        gst = ((d, T2 * d), (d, T2 * d), (2 * d, T2 * 2 * d), (2 * d, T2 * 2 * d))

        def make_train():
            qkv = (torch.randn(rows, 3 * d, device="cuda", generator=gen) * 0.5).bfloat16()
            o = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
            o_lo = torch.empty_like(o)
            do = (torch.randn(rows, d, device="cuda", generator=gen) * 0.1).bfloat16()
            dq = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
            dkv = torch.empty(rows, 2 * d, device="cuda", dtype=torch.bfloat16)
            dm = K.dropmask_buffer(B, H, T2, T2, dh, 0.1, "cuda")
            state = {}

            def fwd():
                state["lse"] = K.attention_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], o, B, H, T2, T2, dh, st, d ** -0.5,
                                               MaskSpec(), 0.1, 77, dropmask=dm, o_lo=o_lo)

            def bwd():
                K.attention_bwd(qkv, qkv[:, d:], qkv[:, 2 * d:], o, state["lse"], do, dq, dkv, dkv[:, d:], B, H, T2,
                                T2, dh, st, gst, d ** -0.5, MaskSpec(), 0.1, 77, dropmask=dm, o_lo=o_lo)
            return fwd, bwd
        nsets = max(2, -(-COLD_BYTES // (rows * d * 14)))
        pairs = [make_train() for _ in range(nsets)]
        tf_ms = _graph_time_ms([f for f, _ in pairs])
        for f, _ in pairs:
            f()
        tb_ms = _graph_time_ms([b_ for _, b_ in pairs])
        for key, t, fl, note in (("attention_fwd_train", tf_ms, flops, "dropout 0.1, O rounding residual"),
                                 ("attention_bwd", tb_ms, 2.5 * flops, "dropout 0.1; FLOPs counted as 2.5x fwd")):
            tt = fl / (t * 1e-3) / 1e12
            out["c5"][key] = {"bound": "mfma", "achieved": round(tt, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                              "frac": round(tt / PEAK_BF16_TFLOPS, 4), "us": round(t * 1e3, 2),
                              "shape": f"B*H={B * H} Lq=Lk={T2} dh={dh}, no mask, training: {note}"}
        del pairs
        torch.cuda.empty_cache()
    return out


def _free_port():
    import socket
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def launch_ranks(nproc, argv, extra_env=None):
    """`--gpus N > 1` without a launcher (no WORLD_SIZE in the environment): start N ranks of this script as a
    CHILD `torch.distributed.run` (this parent process never touches the GPU and never execs), relay rank 0's
    JSON line to stdout, return the child's exit code (non-zero also when no JSON line came back)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra_env or {})
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout.splitlines():
        ln = ln.strip()
        if ln.startswith("{") and ln.endswith("}"):
            line = ln
        else:
            print(ln, file=sys.stderr)
    if line is not None:
        print(line, flush=True)
    if proc.returncode != 0:
        return proc.returncode
    return 0 if line is not None else 1


def cpu_dist_selftest(args, world, rank):
    """Hidden `--cpu-dist-selftest`: the rank/timing/aggregation skeleton of main() on CPU over gloo (no GPU): a
    barrier-bracketed timed loop of trivial steps, max over ranks, one JSON line from rank 0 with n_gpus = world.
    Lets a CPU test drive the `--gpus N` launcher end to end."""
    dist.init_process_group("gloo")
    x = torch.ones(1 << 12)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(x)
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "cpu-dist-selftest", "value": args.steps * world / float(dt), "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # python bench.py --gpus N: spawn the N ranks ourselves (child process), relay rank 0's line
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.cpu_dist_selftest:
        cpu_dist_selftest(args, world, rank)
        return
    torch.cuda.set_device(local)
    # ASRX_DP_REHEARSE=1 at one GPU: a one-rank RCCL group and the data-parallel step path (gradient exchange
    # between captured backward segments, barriers, max-over-ranks timing), so it runs on a 1-GPU box too
    rehearse = world == 1 and os.environ.get("ASRX_DP_REHEARSE", "0") == "1"
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif rehearse:
        os.environ["ASRX_DP_FORCE"] = "1"
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", local))
    dp = world > 1 or rehearse
    import asrx
    from asrx import kernels as K
    from asrx.train import GRAPH_WARMUP, Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch

    spec = CONFIGS[args.config]
    cfg = spec["cfg"]
    B = args.batch or spec["batch"]
    T, L = spec["frames"], spec["text_len"]
    torch.manual_seed(0)
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    if dp:   # identical initial weights on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    trainer = Trainer(model, lr=1e-4, graph=not args.no_graph)
    s, t, m = synthetic_batch(cfg, B, T, L + 1, seed=1234 + rank)
    s, t, m = s.cuda(), t.cuda(), m.cuda()

    # Warm-up.  The last eager step (steady state: gradients bound, unzeroed Linear-weight gradients) times every
    # GEMM launch to find the dominant kernel instantiation; from then on the probe times only that kernel (in
    # graph mode the capture gives it a graph segment of its own, bracketed by HIP events at every replay).  The
    # step is captured as HIP graph(s) at step GRAPH_WARMUP; if the requested warm-up is shorter, the missing
    # steps run untimed as setup (reported as setup_steps).
    probe = None
    setup = 0 if args.no_graph else max(0, GRAPH_WARMUP + 1 - args.warmup)
    survey = args.warmup - 1 if args.no_graph else GRAPH_WARMUP - 1
    for i in range(args.warmup + setup):
        if not args.no_probe and i == survey:
            K.PROBE = K.KernelProbe()
            K.PROBE.active = True
        loss = trainer.step(s, t, m)
        if not args.no_probe and i == survey:
            torch.cuda.synchronize()
            probe = K.KernelProbe(K.PROBE.dominant())
            probe.active = True
            K.PROBE = probe
    torch.cuda.synchronize()
    if probe is not None:
        probe.events = {}
        probe.flops = {}
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    if dp:
        trainer.ar_events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(s, t, m)
    t_enq = time.perf_counter() - t0      # host time to enqueue the K steps (the GPU runs behind it)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    dt = time.perf_counter() - t0
    K.PROBE = None
    if dp:
        x = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        dt = float(x)
    exposed = None
    if dp and trainer.ar_events:
        mine = sum(a.elapsed_time(b) for a, b in trainer.ar_events) / len(trainer.ar_events)
        x = torch.tensor([mine], device="cuda", dtype=torch.float64)
        allv = [torch.zeros_like(x) for _ in range(world)]
        dist.all_gather(allv, x)
        exposed = [round(float(v), 3) for v in allv]
    frames = B * T * args.steps * world
    value = frames / dt
    roof = None
    if probe is not None and probe.events.get(probe.target):
        durs = probe.durations_ms(probe.target)
        avg_ms = sum(durs) / len(durs)
        achieved = probe.flops[probe.target] / (sum(durs) * 1e-3) / 1e12
        per_step = len(durs) // args.steps
        flop_launch = probe.flops[probe.target] // len(durs)
        # the committed PMC summaries are per launch of the single-GPU step; with the data-parallel release
        # schedule the grouped weight-gradient kernel runs as several smaller launches, where they do not apply:
        # use them only when the profiled launch did the same work (MFMA FLOP within 2 %)
        pm = pmc_mfma(probe.target, args.config)
        same = bool(pm and pm.get("mfma_flop_per_launch") and
                    abs(pm["mfma_flop_per_launch"] / flop_launch - 1.0) < 0.02)
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                "traffic": pmc_traffic(probe.target, args.config) if same else None,
                "kernel": probe.target, "launches_per_step": per_step,
                "avg_launch_us": round(avg_ms * 1e3, 2),
                "flop_per_launch_avg": flop_launch,
                "pmc_mfma": pm if same else None}
        if not same:
            roof["pmc_note"] = "traffic / pmc_mfma omitted: no committed PMC profile of a launch of this size"
        ab = probe.alg_bytes.get(probe.target)
        if ab:
            # the launch is on both roofs at once (GEMM FLOPs on the matrix unit, operand panels + dW + fused optimizer
            # state through HBM): its floor is the larger of the two times, frac = floor / measured time
            t_mfma, t_hbm = flop_launch / (PEAK_BF16_TFLOPS * 1e12), ab / (PEAK_HBM_GBS * 1e9)
            roof["combined"] = {"alg_bytes_per_launch": ab, "mfma_floor_us": round(t_mfma * 1e6, 1),
                                "hbm_floor_us": round(t_hbm * 1e6, 1),
                                "frac": round(max(t_mfma, t_hbm) / (avg_ms * 1e-3), 4),
                                "note": "max(FLOP / dense bf16 peak, algorithmic bytes / HBM peak) / launch time"}
        cover = getattr(trainer, "_cover", None)
        if probe.target in K.GROUPED_FUSED_KERNELS and cover:
            n_opt = sum(k for _, k in cover)
            roof["fused_optimizer"] = {
                "op": "AdamW", "params": n_opt, "bytes_per_launch": 26 * n_opt,
                "note": "the launch also runs the optimizer step of these parameters in its epilogue (fp32 master, "
                        "both moments, bf16 shadow: 26 B each beyond the GEMM's own dW store); achieved / frac count "
                        "the GEMM FLOPs only, traffic includes the optimizer bytes"}
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
           "graph": trainer._cap is not None, "setup_steps": setup,
           "allreduce_exposed_ms_per_rank": exposed, "grad_wire": trainer.reducer.wire if dp else None,
           "dp_rehearsal": rehearse,
           "loss": round(float(loss), 4),
           "roofline": roof}
    if rank == 0 and not args.no_sub:
        out["sub_rooflines"] = sub_rooflines(B, asrx.subsampled(T), cfg.d_model, cfg.n_heads, cfg.ff_dim,
                                             cfg.dropout)
    if rank == 0 and world == 1 and not args.no_other:
        out["other_configs"] = other_configs()
        try:   # (a supplementary line: an error here must not cost the headline its JSON line)
            out["other_configs"]["new_small"] = new_train_step()
        except Exception as ex:   # noqa: BLE001
            out["other_configs"]["new_small"] = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, T, L, args.cpu_batch, args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
