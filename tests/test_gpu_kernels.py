"""Per-kernel numerics of libasrx.so on the GPU vs plain PyTorch fp32/fp64 references."""
import math

import numpy as np

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import asrx
    asrx.native()


def K():
    from asrx import kernels
    return kernels


def relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def bf(x):
    return x.to(torch.bfloat16)


# ------------------------------------------------------------------------------------------------ GEMM

VARIANTS = ["auto", "p3", "p4", "reg", "ring", "ring128"]   # kernel families the auto plan can select (gemm.hip plan_bf16)


@pytest.fixture
def kernel_variant(request, monkeypatch):
    """Force a GEMM kernel family (asrx_gemm_desc.kernel) for every gemm() call of the test."""
    monkeypatch.setattr(K(), "GEMM_KERNEL", K().KERNEL_CODES[request.param])
    return request.param


@pytest.mark.parametrize("kernel_variant,tile,dtype", [(v, 0, torch.bfloat16) for v in VARIANTS] +
                         [("reg", 128, torch.bfloat16), ("auto", 0, torch.float32)], indirect=["kernel_variant"])
@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("m,n,k", [(200, 136, 96), (1000, 250, 64), (129, 64, 576), (64, 1536, 512), (33, 17, 40),
                                   (264, 392, 1216), (300, 512, 128)])
def test_gemm_layouts(dtype, at, bt, m, n, k, tile, kernel_variant):
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n * 3 + k)
    A = torch.randn(m, k, generator=g)
    B = torch.randn(n, k, generator=g)
    Ad = (A.t().contiguous() if at else A).to(dev, dtype)
    Bd = (B.t().contiguous() if bt else B).to(dev, dtype)
    C = torch.empty(m, n, device=dev, dtype=torch.float32)
    K().gemm(Ad, Bd, C, m, n, k, lda=Ad.stride(0), ldb=Bd.stride(0), ldc=n, a_trans=at, b_trans=bt,
             tile=tile if dtype == torch.bfloat16 else 0)
    ref = A.to(dtype).double() @ B.to(dtype).double().t()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert relerr(C.cpu(), ref) < tol


@pytest.mark.parametrize("kernel_variant", VARIANTS, indirect=True)
@pytest.mark.parametrize("tile", [64, 128])
def test_gemm_epilogue(tile, kernel_variant):
    m, n, k = 300, 192, 128
    g = torch.Generator().manual_seed(1)
    x = torch.randn(m, k, generator=g)
    w = torch.randn(n, k, generator=g) * 0.1
    bias = torch.randn(n, generator=g)
    pe = torch.randn(50, n, generator=g)
    res = torch.randn(m, n, generator=g)
    gate = torch.randn(m, n, generator=g)
    out = torch.empty(m, n, device=dev)
    K().gemm(bf(x).to(dev), bf(w).to(dev), out, m, n, k, lda=k, ldb=k, ldc=n, alpha=0.5, bias=bias.to(dev),
             rowadd=pe.to(dev), rowadd_mod=50, ld_rowadd=n, relu=True, gate=gate.to(dev), ld_gate=n,
             resid=res.to(dev), ld_resid=n, tile=tile)
    acc = 0.5 * (bf(x).double() @ bf(w).double().t()) + bias.double() + pe.double()[torch.arange(m) % 50]
    ref = torch.where(gate > 0, acc.clamp_min(0), torch.zeros(())) + res.double()
    assert relerr(out.cpu(), ref) < 2e-3


@pytest.mark.parametrize("kernel_variant", ["auto", "p3", "p4", "ring", "ring128"], indirect=True)
@pytest.mark.parametrize("m,n,p", [(300, 512, 0.1), (1000, 4160, 0.0), (4096, 2048, 0.1)])
def test_gemm_relu_mask_bits(m, n, p, kernel_variant):
    """FFN hidden layer: the ReLU/dropout epilogue also writes the 1-bit mask C > 0 (mask_out), and the data
    gradient gated by those bits (gate_bits) equals the one gated by the bf16 C itself, bit for bit."""
    k = 256
    g = torch.Generator(device=dev).manual_seed(m + n)
    x = bf(torch.randn(m, k, device=dev, generator=g))
    w = bf(torch.randn(n, k, device=dev, generator=g) * 0.1)
    bias = torch.randn(n, device=dev, generator=g) * 0.1
    f = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    f0 = torch.empty_like(f)
    bits = torch.full((m, n // 32 + 3), -1, device=dev, dtype=torch.int32)   # padded rows: strays would show
    K().linear(x, w, f, bias=bias, relu=True, dropout_p=p, seed=77, mask_out=bits, ld_mask=n // 32 + 3)
    K().linear(x, w, f0, bias=bias, relu=True, dropout_p=p, seed=77)
    torch.cuda.synchronize()
    assert torch.equal(f, f0)
    pos = (f.float() > 0).view(m, n // 32, 32).to(torch.int64)
    c = torch.arange(32, device=dev)
    want = (pos << (8 * ((c & 15) >> 2) + 4 * (c >> 4) + (c & 3))).sum(-1)   # include/asrx.h mask_out layout
    got = bits[:, :n // 32].to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(got, want)
    assert bool((bits[:, n // 32:] == -1).all())
    dy = bf(torch.randn(m, k, device=dev, generator=g))
    wt = w.t().contiguous()
    for alpha in (1.0, 1.0 / 0.9):
        d_bits = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        d_gate = torch.empty_like(d_bits)
        K().linear_dgrad(dy, wt, d_bits, alpha=alpha, gate=bits, ld_gate=n // 32 + 3,
                         gate_bits=True)
        K().linear_dgrad(dy, wt, d_gate, alpha=alpha, gate=f, ld_gate=n)
        torch.cuda.synchronize()
        assert torch.equal(d_bits, d_gate)
        ref = torch.where(f.float() > 0, alpha * (dy.float() @ wt.float()), torch.zeros((), device=dev))
        assert relerr(d_bits.float(), ref) < 1e-2


def test_gemm_mask_out_unsupported():
    """mask_out needs relu and the paired bf16 store epilogue: fp32 C, N % 32 != 0 or no relu is refused, not
    silently skipped."""
    x = bf(torch.randn(64, 64, device=dev))
    w = bf(torch.randn(48, 64, device=dev))
    bits = torch.zeros(64, 2, device=dev, dtype=torch.int32)
    with pytest.raises(Exception):
        K().linear(x, w, torch.empty(64, 48, device=dev, dtype=torch.bfloat16), relu=True, mask_out=bits, ld_mask=2)
    w = bf(torch.randn(64, 64, device=dev))
    with pytest.raises(Exception):
        K().linear(x, w, torch.empty(64, 64, device=dev), relu=True, mask_out=bits, ld_mask=2)
    with pytest.raises(Exception):   # the bits are the ReLU mask: without relu the request is refused
        K().linear(x, w, torch.empty(64, 64, device=dev, dtype=torch.bfloat16), mask_out=bits, ld_mask=2)


def test_gemm_beta_splitk_and_bf16_out():
    m, n, k = 64, 96, 5000
    g = torch.Generator().manual_seed(2)
    A = torch.randn(k, m, generator=g)            # stored [K][M] -> a_trans
    B = torch.randn(k, n, generator=g)            # stored [K][N] -> b_trans
    C0 = torch.randn(m, n, generator=g)
    C = C0.clone().to(dev)
    K().gemm(bf(A).to(dev), bf(B).to(dev), C, m, n, k, lda=m, ldb=n, ldc=n, a_trans=True, b_trans=True, beta=1.0,
             splitk=7)
    ref = C0.double() + bf(A).double().t() @ bf(B).double()
    assert relerr(C.cpu(), ref) < 2e-3
    Cb = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    K().gemm(bf(A).to(dev), bf(B).to(dev), Cb, m, n, k, lda=m, ldb=n, ldc=n, a_trans=True, b_trans=True)
    assert relerr(Cb.float().cpu(), ref - C0.double()) < 1e-2


@pytest.mark.parametrize("kernel_variant", ["auto", "p3", "reg"], indirect=True)
@pytest.mark.parametrize("tile,splitk", [(64, 1), (128, 1), (64, 5), (128, 7)])
def test_gemm_fused_rowsum(tile, splitk, kernel_variant):
    """wgrad GEMM dW = dY^T X with the bias gradient (row sums of dY^T) fused into the staging/fragments."""
    rows, n_out, k_in = 2048, 384, 256
    g = torch.Generator().manual_seed(tile + splitk)
    dy = bf(torch.randn(rows, n_out, generator=g))
    x = bf(torch.randn(rows, k_in, generator=g))
    wg = torch.ones(n_out, k_in, device=dev)
    bg = torch.full((n_out,), 2.0, device=dev)
    K().gemm(dy.to(dev), x.to(dev), wg, n_out, k_in, rows, lda=n_out, ldb=k_in, ldc=k_in, a_trans=True,
             b_trans=True, beta=1.0, tile=tile, splitk=splitk, rowsum=bg)
    assert relerr(wg.cpu(), 1 + dy.double().t() @ x.double()) < 2e-3
    assert relerr(bg.cpu(), 2 + dy.double().sum(0)) < 1e-5


@pytest.mark.parametrize("wkind,xcd", [("reg", False), ("reg", True), ("p3", False), ("p3", True), ("p4", False),
                                       ("p4", True), ("ws", False), ("ws", True), ("wsq", False), ("wsq", True)])
@pytest.mark.parametrize("ngroups", [1, 7, 60])
def test_gemm_grouped_wgrad(ngroups, wkind, xcd, monkeypatch):
    """Grouped weight gradients (asrx_gemm_grouped_xcd): ragged shapes, K not a multiple of 64, fused bias-grad
    row sums, beta=1 accumulation into existing fp32 grads, 60 problems in one launch (device table written by
    asrx_upload, > 1 chunk).  wsq: the ws tiles from persistent workgroups on per-XCD queues (ws: one workgroup
    per tile)."""
    g = torch.Generator(device=dev).manual_seed(ngroups)
    shapes = [(1000, 136, 96), (4096, 512, 512), (333, 248, 64), (64, 8, 576), (2500, 1536, 512),
              (77, 40, 1216), (249, 200, 24)]
    monkeypatch.setattr(K(), "WGRAD_KIND", "ws" if wkind == "wsq" else wkind)
    monkeypatch.setattr(K(), "WGRAD_QUEUE", wkind == "wsq")
    monkeypatch.setattr(K(), "WGRAD_XCD", xcd)
    items, refs = [], []
    for i in range(ngroups):
        M, N, Kd = shapes[i % len(shapes)]
        dy = bf(torch.randn(M, N, device=dev, generator=g))
        x = bf(torch.randn(M, Kd, device=dev, generator=g))
        wg = torch.randn(N, Kd, device=dev, generator=g)
        bg = torch.randn(N, device=dev, generator=g) if i % 2 == 0 else None
        refs.append((wg + dy.float().t() @ x.float(), None if bg is None else bg + dy.float().sum(0)))
        items.append((dy, x, wg, bg))
    kname = K().linear_wgrad_grouped(items)
    torch.cuda.synchronize()
    if wkind == "wsq" and xcd:
        assert kname.startswith("gemm_bf16_wsgq_kernel"), kname   # the queue kernel ran
    elif wkind in ("ws", "wsq"):
        assert kname.startswith(("gemm_bf16_wsg_kernel", "gemm_bf16_wsgq_kernel")), kname
        assert wkind == "wsq" or kname.startswith("gemm_bf16_wsg_kernel"), kname
    odd = bf(torch.randn(10, 250, device=dev))      # rows not 16-byte aligned: not groupable (C.wgrad runs it alone)
    assert not K().wgrad_groupable(odd, bf(torch.randn(10, 64, device=dev)), torch.zeros(250, 64, device=dev))
    for (dy, x, wg, bg), (rw, rb) in zip(items, refs):
        assert relerr(wg, rw) < 1e-5, dy.shape
        if bg is not None:
            assert relerr(bg, rb) < 1e-5


@pytest.mark.parametrize("rows,n", [(302784, 576), (40000, 576), (16384 + 37, 128), (70001, 512)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_linear_wgrad_tallk(rows, n, with_bias):
    """conv2-shaped weight gradient dW[64, n] += dy^T x over a very tall reduction (the many-split tall-K kernel,
    plan use 9): ragged split ends, fused bias gradient, beta=1 accumulation."""
    g = torch.Generator(device=dev).manual_seed(rows + n)
    dy = bf(torch.randn(rows, 64, device=dev, generator=g))
    x = bf(torch.randn(rows, n, device=dev, generator=g))
    wg = torch.randn(64, n, device=dev, generator=g)
    bg = torch.randn(64, device=dev, generator=g) if with_bias else None
    ref = wg.double() + dy.double().t() @ x.double()
    rb = None if bg is None else bg.double() + dy.double().sum(0)
    tile, splitk = K().wgrad_plan(64, n, rows)
    assert splitk == 256
    from asrx._lib import GemmDesc
    d = GemmDesc(64, n, rows, 0, dy.data_ptr(), 64, 1, x.data_ptr(), n, 1, wg.data_ptr(), n, 1)
    d.splitk = splitk
    assert K().kernel_name(d) == "gemm_bf16_tallk_kernel"
    K().linear_wgrad(dy, x, wg, bias_grad=bg)
    torch.cuda.synchronize()
    assert relerr(wg, ref) < 1e-5
    if bg is not None:
        assert relerr(bg, rb) < 1e-5


def test_gemm_batched_heads():
    """Two-level batch strides as used by the unfused attention: z = b*H + h."""
    Bn, H, L, dh = 3, 4, 37, 32
    d = H * dh
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(Bn, L, 3 * d, generator=g)
    q = qkv[..., :d].reshape(Bn, L, H, dh).permute(0, 2, 1, 3)
    k = qkv[..., d:2 * d].reshape(Bn, L, H, dh).permute(0, 2, 1, 3)
    ld = 40
    S = torch.zeros(Bn * H, L, ld, device=dev)
    x = qkv.to(dev)
    K().gemm(x, x[..., d:], S, L, L, dh, lda=3 * d, ldb=3 * d, ldc=ld, batch=Bn * H, batch_inner=H,
             sa=(L * 3 * d, dh), sb=(L * 3 * d, dh), sc=(H * L * ld, L * ld))
    ref = (q.double() @ k.double().transpose(-1, -2)).reshape(Bn * H, L, L)
    assert relerr(S[:, :, :L].cpu(), ref) < 1e-5


def plan_name(M, N, Kd, bt=False, bias=False, c_f32=False, resid=False, dropout=False, kernel=0):
    """asrx_gemm_kernel_name of a (M, N, K) GEMM with fake 16-B aligned pointers: the kernel the plan picks."""
    from asrx._lib import BF16, F32, GemmDesc
    from asrx.kernels import KERNEL_CODES, kernel_name
    d = GemmDesc()
    d.m, d.n, d.k, d.in_dtype = M, N, Kd, BF16
    d.a, d.lda = 1 << 20, Kd
    d.b, d.ldb, d.b_trans = 2 << 20, (N if bt else Kd), int(bt)
    d.c, d.ldc, d.c_dtype = 3 << 20, N, (F32 if c_f32 else BF16)
    d.alpha, d.batch, d.batch_inner, d.splitk = 1.0, 1, 1, 1
    d.kernel = KERNEL_CODES.get(kernel, kernel)
    if bias:
        d.bias = 4 << 20
    if resid:
        d.resid, d.ld_resid, d.resid_dtype = 5 << 20, N + 8, F32
    if dropout:
        d.dropout_p = 0.1
    return kernel_name(d)


@pytest.mark.parametrize("wk", ["ws", "ws64"])
@pytest.mark.parametrize("M,N,Kd,bt", [(15936, 512, 2048, 1), (15936, 512, 1536, 1), (300, 256, 192, 1),
                                        (257, 128, 64, 0), (64, 512, 2048, 1), (1000, 384, 640, 0),
                                        (4096, 512, 1536, 1), (4096, 512, 512, 0), (4033, 512, 2048, 1)])
def test_gemm_ws_plain(M, N, Kd, bt, wk):
    """The warp-specialised kernel on 256x128 tiles (kernel code 8; chosen automatically for the encoder's plain
    512-wide data gradients) and on 64x128 tiles (code 10; the decoder's 4096-row ones): C = A . op(B) in bf16
    against an fp64 reference, both B layouts, ragged M (rows past M read as zero, stores masked), and identical to
    the auto plan at the bench shapes."""
    g = torch.Generator().manual_seed(M + N + Kd)
    a = bf(torch.randn(M, Kd, generator=g))
    b = bf(torch.randn(Kd, N, generator=g) if bt else torch.randn(N, Kd, generator=g))
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = a.double() @ (b.double() if bt else b.double().t())
    kn = plan_name(M, N, Kd, bt=bt, kernel=wk)
    assert kn.startswith("gemm_bf16_ws_kernel") and kn.endswith("64>" if wk == "ws64" else "256>"), kn
    K().gemm(a.to(dev), b.to(dev), c, M, N, Kd, lda=Kd, ldb=b.shape[1], ldc=N, b_trans=bool(bt), kernel=wk)
    assert relerr(c.float().cpu(), ref) < 1e-2
    auto_ws = N == 512 and (M >= 8192 if wk == "ws" else 2048 <= M < 8192)
    if bt and auto_ws:   # the auto plan takes the same path
        c2 = torch.empty_like(c)
        K().gemm(a.to(dev), b.to(dev), c2, M, N, Kd, lda=Kd, ldb=N, ldc=N, b_trans=True)
        assert torch.equal(c, c2)


@pytest.mark.parametrize("wk", ["ws", "ws64"])
@pytest.mark.parametrize("M,N,Kd,f32,resid,drop", [(15936, 512, 2048, 1, 1, 0), (4096, 512, 2048, 1, 1, 0),
                                                   (300, 256, 128, 1, 1, 0), (257, 128, 64, 1, 0, 0),
                                                   (257, 128, 64, 0, 0, 0), (15936, 512, 512, 1, 1, 1),
                                                   (700, 384, 256, 1, 1, 1), (4096, 512, 512, 1, 1, 1),
                                                   (4096, 512, 512, 0, 0, 0)])
def test_gemm_ws_bias_resid(M, N, Kd, f32, resid, drop, wk):
    """The ws kernel's LDS-staged epilogue: out = x . w^T + bias (+ dropout) (+ fp32 residual, ld_resid != ldc) —
    the FFN2 forward (E_BIAS | E_RESID | E_F32) and the out-projection (+ E_DROP) — forced (kernel code 8) against
    an fp64 reference, and element-for-element against the p3 epilogue on the same inputs (same keep bits; fp32
    accumulation-order differences only)."""
    g = torch.Generator().manual_seed(M + 3 * N + Kd)
    x, w = bf(torch.randn(M, Kd, generator=g)), bf(torch.randn(N, Kd, generator=g))
    bias = torch.randn(N, generator=g)
    r = torch.randn(M, N + 8, generator=g) if resid else None   # ld_resid = N + 8 != ldc
    ref = x.double() @ w.double().t() + bias.double()
    kw = dict(resid=r.to(dev), ld_resid=N + 8) if resid else {}
    if drop:
        kw.update(dropout_p=0.1, seed=77)
    outs = {}
    for kern in ("ws", "p3"):
        c = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        K().linear(x.to(dev), w.to(dev), c, bias=bias.to(dev), kernel=wk if kern == "ws" else kern, **kw)
        outs[kern] = c.float().cpu()
    kn = plan_name(M, N, Kd, bias=True, c_f32=bool(f32), resid=bool(resid), dropout=bool(drop), kernel=wk)
    assert kn.startswith("gemm_bf16_ws_kernel") and kn.endswith("64>" if wk == "ws64" else "256>"), kn
    if drop:   # same keep bits in both kernels; the reference is p3's kept pattern
        keep = (outs["p3"] - (r[:, :N] if resid else 0)) != 0
        ref = torch.where(keep, ref / 0.9, torch.zeros_like(ref))
    if resid:
        ref = ref + r[:, :N].double()
    for kern, o in outs.items():
        assert relerr(o, ref) < (1e-5 if f32 else 1e-2), kern
    assert (outs["ws"] - outs["p3"]).abs().max() <= (1e-4 if f32 else 1e-2) * ref.abs().max()


def test_gemm_ws_rowadd():
    """The ws kernel's row-periodic add (E_ROWADD, the _lin_in GEMM's positional-encoding epilogue: row m takes
    table row m % T'), fp32 out, against fp64 and against p3."""
    M, N, Kd, T2 = 15936, 512, 1216, 249
    g = torch.Generator().manual_seed(11)
    x, w = bf(torch.randn(M, Kd, generator=g)), bf(torch.randn(N, Kd, generator=g))
    bias, pe = torch.randn(N, generator=g), torch.randn(T2, N, generator=g)
    ref = x.double() @ w.double().t() + bias.double() + pe.double().repeat(M // T2 + 1, 1)[:M]
    outs = {}
    for kern in ("ws", "p3"):
        c = torch.empty(M, N, device=dev)
        K().gemm(x.to(dev), w.to(dev), c, M, N, Kd, lda=Kd, ldb=Kd, ldc=N, bias=bias.to(dev), rowadd=pe.to(dev),
                 rowadd_mod=T2, ld_rowadd=N, kernel=kern)
        outs[kern] = c.cpu()
        assert relerr(outs[kern], ref) < 1e-5, kern
    assert (outs["ws"] - outs["p3"]).abs().max() <= 1e-4 * ref.abs().max()


@pytest.mark.parametrize("B,H,L,Lk", [(64, 8, 249, 249), (64, 8, 64, 64), (64, 8, 64, 249), (3, 2, 37, 37),
                                      (3, 2, 37, 300)])
def test_layernorm_fused_with_keep_bits(B, H, L, Lk):
    """asrx_layernorm_fwd_attn_dropgen: the LayerNorm part equals asrx_layernorm_fwd bit for bit and the keep bits
    (both layouts) equal asrx_attn_dropgen's, for the encoder (249 keys), the decoder self (64) and cross (64
    queries over the 249 encoder frames: rows = B x queries) attention, and ragged shapes."""
    d = 512
    rows = B * L
    g = torch.Generator(device=dev).manual_seed(rows)
    x = torch.randn(rows, d, device=dev, generator=g) * 2 + 0.3
    gam = torch.rand(d, device=dev, generator=g) + 0.5
    bet = torch.randn(d, device=dev, generator=g)
    y1 = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y1)
    m1, r1 = K().layernorm_fwd(x, gam, bet, y1)
    dm1 = K().dropmask_buffer(B, H, L, Lk, 64, 0.1, dev)
    dm2 = K().dropmask_buffer(B, H, L, Lk, 64, 0.1, dev)
    K().attention_dropgen(B, H, L, Lk, 64, 0.1, 1234567, dm1)
    m2, r2 = K().layernorm_fwd_dropgen(x, gam, bet, y2, B, H, L, Lk, 64, 0.1, 1234567, dm2)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2) and torch.equal(m1, m2) and torch.equal(r1, r2)
    assert torch.equal(dm1, dm2)


# ------------------------------------------------------------------------------------------------ LayerNorm

@pytest.fixture
def tuning():
    """Set a kernel-variant switch (asrx_set_tuning) for one test and restore the default afterwards."""
    used = []

    def set_(name, value):
        used.append(name)
        K().set_tuning(name, value)
    yield set_
    for name in used:
        K().set_tuning(name, 0)


@pytest.mark.parametrize("d", [64, 128, 256, 512])
@pytest.mark.parametrize("ydt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rw,pf", [(0, 0), (1, 8), (4, 8), (2, 8), (0, 1), (0, 4)])
@pytest.mark.parametrize("rows", [333, 15936])
@pytest.mark.parametrize("dyt", [torch.float32, torch.bfloat16])
def test_layernorm(d, ydt, rw, pf, rows, dyt, tuning):
    """rw: rows per wave of the general forward (0 = default 2; 1 and 4 the other variants); pf: rows in
    flight per wave of the d = 512 streaming kernels (0 = default 2; 8 = the general kernels); dyt: the incoming
    gradient's dtype (bf16: the compute dtype of the layers; fp32: the encoder's final LayerNorm, fed by the fp32
    cross K/V data gradient — both on the d = 512 kernel since round 6)."""
    tuning("ln_rw", rw)
    tuning("ln_pf", pf)
    if rows > 1000 and (d != 512 or rw != 0):
        pytest.skip("the bench-size row count only for the d = 512 streaming variants")
    if dyt == torch.bfloat16 and (ydt == torch.float32 or rw != 0):
        pytest.skip("bf16 dy: one forward variant suffices")
    g = torch.Generator().manual_seed(d)
    x = torch.randn(rows, d, generator=g) * 2 + 0.5
    gam = 1 + 0.1 * torch.randn(d, generator=g)
    bet = 0.1 * torch.randn(d, generator=g)
    dy = torch.randn(rows, d, generator=g).to(dyt)
    dres = torch.randn(rows, d, generator=g)
    y = torch.empty(rows, d, device=dev, dtype=ydt)
    mean, rstd = K().layernorm_fwd(x.to(dev), gam.to(dev), bet.to(dev), y)
    xr = x.double().requires_grad_(True)
    gr = gam.double().requires_grad_(True)
    br = bet.double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (d,), gr, br, 1e-5)
    assert relerr(y.float().cpu(), yr.detach()) < (1e-5 if ydt == torch.float32 else 1e-2)
    yr.backward(dy.double())   # (bf16 dy: the reference sees the same rounded values)
    dgb = torch.zeros(2 * d, device=dev)
    drop = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
    dx = K().layernorm_bwd(x.to(dev), dy.to(dev), gam.to(dev), mean, rstd, dgb, dres=dres.to(dev), dx_drop=drop)
    assert relerr(dx.cpu(), xr.grad + dres.double()) < 1e-5
    assert relerr(drop.float().cpu(), xr.grad + dres.double()) < 1e-2
    assert relerr(dgb[:d].cpu(), gr.grad) < 1e-5
    assert relerr(dgb[d:].cpu(), br.grad) < 1e-5


@pytest.mark.parametrize("ngroups", [1, 70])
def test_reduce_rows_grouped(ngroups):
    """Deferred LayerNorm partial reductions: many fp32 matrices' column sums in grouped launches."""
    g = torch.Generator(device=dev).manual_seed(ngroups)
    items, refs = [], []
    for i in range(ngroups):
        rows, cols = [(512, 1024), (3, 70), (1, 64), (129, 256)][i % 4]
        x = torch.randn(rows, cols, device=dev, generator=g)
        out = torch.randn(cols, device=dev, generator=g)
        acc = i % 3 != 0
        refs.append((out.double() if acc else 0) + x.double().sum(0))
        items.append((x, out, acc))
    K().reduce_rows_grouped(items)
    torch.cuda.synchronize()
    for (x, out, acc), r in zip(items, refs):
        assert relerr(out, r) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_ewise(dt):
    """asrx_ewise vs torch: ReLU gate, dropout backward (the element mask of asrx_dropout_mask / the GEMM dropout
    epilogues), add; mixed dtypes and in-place outputs."""
    g = torch.Generator(device=dev).manual_seed(3)
    n = 100_003
    a = torch.randn(n, device=dev, generator=g).to(dt)
    b = torch.randn(n, device=dev, generator=g).to(dt)
    out = torch.empty(n, device=dev, dtype=torch.float32)
    K().ewise(K().EW_RELU_GRAD, a, out, b=b)
    assert torch.equal(out, torch.where(b > 0, a, torch.zeros((), dtype=dt, device=dev)).float())
    p, seed = 0.1, 12345
    K().ewise(K().EW_DROPOUT, a, out, p=p, seed=seed)
    keep = K().dropout_mask(n, p, seed, dev)
    assert torch.allclose(out, a.float() * keep / (1 - p), rtol=1e-6, atol=0)
    c = a.clone()
    K().ewise(K().EW_ADD, c, c, b=b)
    assert torch.equal(c, (a.float() + b.float()).to(dt))


def test_colsum():
    x = torch.randn(10000, 300)
    out = torch.ones(300, device=dev)
    K().colsum(x.to(dev), out)
    assert relerr(out.cpu(), x.double().sum(0) + 1) < 1e-5


# ------------------------------------------------------------------------------------------------ attention

def ref_attention(q, k, v, scale, masked, p_keep=None):
    """q (B,H,Lq,dh) etc. in fp64; masked bool (B,1|H,Lq,Lk); reference semantics layers.py:20-27."""
    s = (q @ k.transpose(-1, -2)) * scale
    s = s.masked_fill(masked, float("-inf"))
    p = torch.nan_to_num(torch.softmax(s, -1))
    pd = p if p_keep is None else p * p_keep
    return pd @ v, p


def _mk(B, H, Lq, Lk, dh, kind, g):
    d = H * dh
    q = torch.randn(B, Lq, d, generator=g)
    kv = torch.randn(B, Lk, 2 * d, generator=g)
    valid = torch.ones(B, max(Lq, Lk))
    if kind == "decoder":
        valid[0, Lq // 2:] = 0
        valid[-1, 2:] = 0
    return q, kv, valid


def _masked(kind, B, Lq, Lk, valid):
    if kind == "none":
        return torch.zeros(B, 1, Lq, Lk, dtype=torch.bool)
    pad = valid[:, :Lk].lt(1).unsqueeze(1).expand(-1, Lq, -1)
    m = pad | pad.transpose(1, 2) | torch.triu(torch.ones(Lq, Lk, dtype=torch.bool), 1)
    return m.unsqueeze(1)


@pytest.fixture
def attn_variant(request):
    import os
    old = os.environ.get("ASRX_ATTN_KERNEL")
    os.environ["ASRX_ATTN_KERNEL"] = request.param
    yield request.param
    if old is None:
        os.environ.pop("ASRX_ATTN_KERNEL", None)
    else:
        os.environ["ASRX_ATTN_KERNEL"] = old


@pytest.mark.parametrize("attn_variant", ["auto", "tiled", "resident"], indirect=True)
@pytest.mark.parametrize("dh", [32, 64])
@pytest.mark.parametrize("B,H,Lq,Lk,kind", [(2, 4, 70, 70, "decoder"), (3, 2, 64, 249, "none"),
                                           (2, 2, 249, 249, "none"), (1, 2, 100, 300, "none"),
                                           (2, 3, 33, 33, "decoder"), (1, 2, 300, 64, "none"),
                                           (2, 2, 256, 256, "decoder"), (1, 1, 5, 17, "none"),
                                           (1, 2, 999, 999, "none"), (1, 2, 300, 300, "decoder"),
                                           (1, 2, 64, 257, "none"), (2, 2, 513, 1031, "none"),
                                           (2, 2, 100, 200, "none"), (1, 3, 249, 240, "none"),
                                           (2, 2, 64, 100, "none"), (2, 3, 33, 256, "none")])
def test_attention_fused(dh, B, H, Lq, Lk, kind, attn_variant):
    from asrx.kernels import MaskSpec
    g = torch.Generator().manual_seed(B * 100 + Lq + Lk + dh)
    q, kv, valid = _mk(B, H, Lq, Lk, dh, kind, g)
    d = H * dh
    qb, kvb = bf(q), bf(kv)
    qd, kvd = qb.to(dev), kvb.to(dev)
    o = torch.empty(B * Lq, d, device=dev, dtype=torch.bfloat16)
    if kind == "decoder":
        vv = (valid[:, :Lq] >= 1).to(torch.uint8).to(dev)
        spec = MaskSpec(1, True, vv, vv, vv.stride(0))
    else:
        spec = MaskSpec()
    scale = (d) ** -0.5
    st = ((d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d), (d, Lq * d))
    lse = K().attention_fwd(qd, kvd, kvd[..., d:], o, B, H, Lq, Lk, dh, st, scale, spec)
    qh = qb.double().view(B, Lq, H, dh).transpose(1, 2).requires_grad_(True)
    kh = kvb[..., :d].double().reshape(B, Lk, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    vh = kvb[..., d:].double().reshape(B, Lk, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    masked = _masked(kind, B, Lq, Lk, valid)
    ref, _ = ref_attention(qh, kh, vh, scale, masked)
    out = o.float().cpu().view(B, Lq, H, dh).transpose(1, 2)
    assert relerr(out, ref.detach()) < 1e-2
    if kind == "decoder":
        # fully-masked query rows (query padding) are exactly zero (nan_to_num, layers.py:25)
        rows = (valid[:, :Lq] < 1)
        assert torch.all(out.permute(0, 2, 1, 3)[rows] == 0)
    # backward
    dO = torch.randn(B, Lq, d, generator=g)
    dOb = bf(dO)
    ref.backward(dOb.double().view(B, Lq, H, dh).transpose(1, 2))
    dq = torch.empty(B * Lq, d, device=dev, dtype=torch.bfloat16)
    dkv = torch.empty(B * Lk, 2 * d, device=dev, dtype=torch.bfloat16)
    gst = ((d, Lq * d), (d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d))
    K().attention_bwd(qd, kvd, kvd[..., d:], o, lse, dOb.to(dev), dq, dkv, dkv[:, d:], B, H, Lq, Lk, dh, st, gst,
                      scale, spec)
    dq_ = dq.float().cpu().view(B, Lq, H, dh).transpose(1, 2)
    dk_ = dkv[:, :d].float().cpu().view(B, Lk, H, dh).transpose(1, 2)
    dv_ = dkv[:, d:].float().cpu().view(B, Lk, H, dh).transpose(1, 2)
    assert relerr(dv_, vh.grad) < 2e-2
    assert relerr(dk_, kh.grad) < 2e-2
    assert relerr(dq_, qh.grad) < 2e-2


@pytest.mark.parametrize("Lq,Lk", [(64, 249), (100, 200), (5, 17), (30, 256), (249, 249), (64, 64), (250, 229),
                                   (64, 999), (300, 300), (257, 520)])
@pytest.mark.parametrize("with_lo", [False, True])
def test_attention_short_query_block_with_dropout(Lq, Lk, with_lo):
    """Short query blocks without a mask (MODE 0, Lq <= 128: the decoder's cross-attention shape) with dropout
    p = 0.3 (keep bits from rng_ref): the output and the saved lse (checked through the backward's gradients) match
    the float64 reference."""
    from asrx.kernels import MaskSpec
    from rng_ref import attn_keep
    B, H, dh = 2, 2, 64
    d = H * dh
    g = torch.Generator().manual_seed(Lq * 1000 + Lk)
    q, kv, valid = _mk(B, H, Lq, Lk, dh, "none", g)
    qb, kvb = bf(q), bf(kv)
    qd, kvd = qb.to(dev), kvb.to(dev)
    st = ((d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d), (d, Lq * d))
    p, seed = 0.3, 4321
    o = torch.empty(B * Lq, d, device=dev, dtype=torch.bfloat16)
    dm = K().dropmask_buffer(B, H, Lq, Lk, dh, p, dev)
    o_lo = torch.empty_like(o) if with_lo else None   # the training path's O rounding residual (exact delta)
    lse = K().attention_fwd(qd, kvd, kvd[..., d:], o, B, H, Lq, Lk, dh, st, d ** -0.5, MaskSpec(), p, seed,
                            dropmask=dm, o_lo=o_lo)
    keep = torch.from_numpy(attn_keep(seed, B * H, Lq, Lk, p)).view(B, H, Lq, Lk).double() / (1 - p)
    qh = qb.double().view(B, Lq, H, dh).transpose(1, 2).requires_grad_(True)
    kh = kvb[..., :d].double().reshape(B, Lk, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    vh = kvb[..., d:].double().reshape(B, Lk, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    ref, _ = ref_attention(qh, kh, vh, d ** -0.5, _masked("none", B, Lq, Lk, valid), keep)
    assert relerr(o.float().cpu().view(B, Lq, H, dh).transpose(1, 2), ref.detach()) < 1e-2
    dO = bf(torch.randn(B, Lq, d, generator=g))
    ref.backward(dO.double().view(B, Lq, H, dh).transpose(1, 2))
    dq = torch.empty(B * Lq, d, device=dev, dtype=torch.bfloat16)
    dkv = torch.empty(B * Lk, 2 * d, device=dev, dtype=torch.bfloat16)
    gst = ((d, Lq * d), (d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d))
    K().attention_bwd(qd, kvd, kvd[..., d:], o, lse, dO.to(dev), dq, dkv, dkv[:, d:], B, H, Lq, Lk, dh, st, gst,
                      d ** -0.5, MaskSpec(), p, seed, dropmask=dm, o_lo=o_lo)
    assert relerr(dq.float().cpu().view(B, Lq, H, dh).transpose(1, 2), qh.grad) < 2e-2
    assert relerr(dkv[:, :d].float().cpu().view(B, Lk, H, dh).transpose(1, 2), kh.grad) < 2e-2
    assert relerr(dkv[:, d:].float().cpu().view(B, Lk, H, dh).transpose(1, 2), vh.grad) < 2e-2


@pytest.mark.parametrize("Lq,Lk", [(249, 249), (64, 249), (57, 1031)])
def test_attention_tensors_at_allocation_end(Lq, Lk):
    """Q, dO, O, O_lo and lse as the LAST bytes of their own device allocations (12 MiB each: torch gives such a
    request a segment of exactly that size), Lq % 32 != 0: the backward's tail chunk must not read past them (ADVICE
    r5 — the round-5 prefetch put the chunk start in the descriptor's soffset, which the range check ignores) and the
    results equal those of ordinary allocations bit for bit (the dQ stores past Lq are dropped by the descriptor)."""
    from asrx.kernels import MaskSpec
    B, H, dh = 1, 2, 64
    d = H * dh
    g = torch.Generator().manual_seed(Lq + 7 * Lk)
    q, kv, _ = _mk(B, H, Lq, Lk, dh, "none", g)
    qb, kvd = bf(q).to(dev), bf(kv).to(dev)
    dO = bf(torch.randn(B, Lq, d, generator=g)).to(dev)
    p, seed, scale = 0.1, 99, d ** -0.5
    st = ((d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d), (d, Lq * d))
    gst = ((d, Lq * d), (d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d))
    seg = 12 << 20

    def tail(n, dtype):   # the last n elements of a fresh 12 MiB allocation
        esz = torch.tensor([], dtype=dtype).element_size()
        return torch.empty(seg // esz, device=dev, dtype=dtype)[-n:]

    def run(at_end):
        q_ = tail(B * Lq * d, torch.bfloat16) if at_end else torch.empty(B * Lq * d, device=dev, dtype=torch.bfloat16)
        q_.copy_(qb.reshape(-1))
        do_ = tail(B * Lq * d, torch.bfloat16) if at_end else torch.empty_like(q_)
        do_.copy_(dO.reshape(-1))
        o = tail(B * Lq * d, torch.bfloat16) if at_end else torch.empty_like(q_)
        o_lo = tail(B * Lq * d, torch.bfloat16) if at_end else torch.empty_like(q_)
        q2, do2, o2, ol2 = (t.view(B * Lq, d) for t in (q_, do_, o, o_lo))
        dm = K().dropmask_buffer(B, H, Lq, Lk, dh, p, dev)
        lse = K().attention_fwd(q2, kvd, kvd[..., d:], o2, B, H, Lq, Lk, dh, st, scale, MaskSpec(), p, seed,
                                dropmask=dm, o_lo=ol2)
        if at_end:
            lt = tail(lse.numel(), torch.float32)
            lt.copy_(lse.reshape(-1))
            lse = lt.view_as(lse)
        dq = torch.empty(B * Lq, d, device=dev, dtype=torch.bfloat16)
        dkv = torch.empty(B * Lk, 2 * d, device=dev, dtype=torch.bfloat16)
        K().attention_bwd(q2, kvd, kvd[..., d:], o2, lse, do2, dq, dkv, dkv[:, d:], B, H, Lq, Lk, dh, st, gst,
                          scale, MaskSpec(), p, seed, dropmask=dm, o_lo=ol2)
        torch.cuda.synchronize()
        return o2.clone(), dq, dkv

    ref = run(False)
    got = run(True)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


@pytest.mark.parametrize("attn_variant", ["auto", "tiled"], indirect=True)
@pytest.mark.parametrize("L", [40, 249, 300])
@pytest.mark.parametrize("bits", [False, True])
def test_attention_dense_mask_and_dropout_consistency(L, attn_variant, bits):
    """Dense byte mask (mode 2) equals the structured decoder mask; the dropout the kernels apply in forward AND
    backward is exactly the keep mask of the numpy RNG restatement (tests/rng_ref.py)."""
    from asrx.kernels import MaskSpec
    from rng_ref import attn_keep, elem_keep
    B, H, dh = 2, 2, 64
    d = H * dh
    g = torch.Generator().manual_seed(9)
    q, kv, valid = _mk(B, H, L, L, dh, "decoder", g)
    qd, kvd = bf(q).to(dev), bf(kv).to(dev)
    masked = _masked("decoder", B, L, L, valid)
    vv = (valid[:, :L] >= 1).to(torch.uint8).to(dev)
    s1 = MaskSpec(1, True, vv, vv, vv.stride(0))
    s2 = MaskSpec.from_attention_mask(masked[:, 0].to(dev), B, L, L)
    st = ((d, L * d), (2 * d, L * 2 * d), (2 * d, L * 2 * d), (d, L * d))
    o1 = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    K().attention_fwd(qd, kvd, kvd[..., d:], o1, B, H, L, L, dh, st, d ** -0.5, s1)
    K().attention_fwd(qd, kvd, kvd[..., d:], o2, B, H, L, L, dh, st, d ** -0.5, s2)
    if L <= 256 or attn_variant == "tiled":   # one kernel for both mask forms
        assert torch.equal(o1, o2)
    else:   # past 256 keys the structured mask streams, a dense byte mask takes the tiled kernel
        assert relerr(o1.float().cpu(), o2.float().cpu()) < 1e-2
        # padded queries: exact zeros
        assert torch.all(o1.view(B, L, d).cpu()[valid[:, :L] < 1] == 0)
        assert torch.all(o2.view(B, L, d).cpu()[valid[:, :L] < 1] == 0)
    p, seed = 0.3, 1234
    o3 = torch.empty_like(o1)
    dm = K().dropmask_buffer(B, H, L, L, dh, p, dev) if bits else None
    lse = K().attention_fwd(qd, kvd, kvd[..., d:], o3, B, H, L, L, dh, st, d ** -0.5, s1, p, seed, dropmask=dm)
    if dm is not None and attn_variant == "auto":   # the forward's published keep bits == the RNG's decisions
        ka = attn_keep(seed, B * H, L, L, p)
        nq = (L + 31) // 32
        words = dm.cpu().numpy().view(np.uint32)[:B * H * nq * L].reshape(B * H, nq, L)
        qst = K().qmaj_stride(L)
        qwords = dm.cpu().numpy().view(np.uint32)[B * H * nq * L:].reshape(B * H, L, qst)
        qbits = (qwords[:, :, :, None] >> np.arange(32, dtype=np.uint32)[None, None, None, :]) & 1
        assert (qbits.reshape(B * H, L, qst * 32)[:, :, :L].astype(bool) == ka).all()   # query-major copy
        bits_np = (words[:, :, None, :] >> np.arange(32, dtype=np.uint32)[None, None, :, None]) & 1
        got = bits_np.reshape(B * H, nq * 32, L)[:, :L, :].astype(bool)
        live = ~masked.expand(B, H, L, L).reshape(B * H, L, L).numpy()   # words of masked-out tiles are never read
        assert (got == ka)[live].all()
    keep = torch.from_numpy(attn_keep(seed, B * H, L, L, p)).view(B, H, L, L).double() / (1 - p)
    em = K().dropout_mask(B * H * L * L, p, seed, dev).cpu().numpy().astype(bool)
    assert (em == elem_keep(seed, B * H * L * L, p)).all()   # element stream bit-exact vs the numpy restatement
    qh = bf(q).double().view(B, L, H, dh).transpose(1, 2).requires_grad_(True)
    kh = bf(kv)[..., :d].double().reshape(B, L, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    vh = bf(kv)[..., d:].double().reshape(B, L, H, dh).transpose(1, 2).contiguous().requires_grad_(True)
    ref, _ = ref_attention(qh, kh, vh, d ** -0.5, masked, keep)
    assert relerr(o3.float().cpu().view(B, L, H, dh).transpose(1, 2), ref.detach()) < 1e-2
    frac = float((keep > 0).double().mean())
    assert abs(frac - (1 - p)) < 0.02
    dO = bf(torch.randn(B, L, d, generator=g))
    ref.backward(dO.double().view(B, L, H, dh).transpose(1, 2))
    dq = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    dkv = torch.empty(B * L, 2 * d, device=dev, dtype=torch.bfloat16)
    gst = ((d, L * d), (d, L * d), (2 * d, L * 2 * d), (2 * d, L * 2 * d))
    K().attention_bwd(qd, kvd, kvd[..., d:], o3, lse, dO.to(dev), dq, dkv, dkv[:, d:], B, H, L, L, dh, st, gst,
                      d ** -0.5, s1, p, seed, dropmask=dm if (dm is not None and attn_variant == "auto") else None)
    assert relerr(dkv[:, d:].float().cpu().view(B, L, H, dh).transpose(1, 2), vh.grad) < 2e-2
    assert relerr(dkv[:, :d].float().cpu().view(B, L, H, dh).transpose(1, 2), kh.grad) < 2e-2
    assert relerr(dq.float().cpu().view(B, L, H, dh).transpose(1, 2), qh.grad) < 2e-2


# ------------------------------------------------------------------------------------------------ softmax

@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Lk", [24, 64, 127, 249, 999])
@pytest.mark.parametrize("u", [0, 2, 4])
def test_softmax_masked(dtype, Lk, u, tuning):
    """u: rows per lane group of the short-row kernels (0 = default 1; 2 and 4 the other variants)."""
    from asrx.kernels import MaskSpec
    tuning("softmax_u", u)
    B, H, Lq = 2, 3, min(Lk, 70)
    g = torch.Generator().manual_seed(Lk)
    ld = (Lk + 7) // 8 * 8
    s = torch.randn(B * H, Lq, ld, generator=g) * 3
    valid = torch.ones(B, Lk)
    valid[1, Lk // 3:] = 0
    vv = (valid >= 1).to(torch.uint8)
    spec = MaskSpec(1, True, vv.to(dev), vv.to(dev), Lk) if Lq == Lk else MaskSpec(1, False, vv.to(dev), None, Lk)
    sd = s.to(dev, dtype)
    p = torch.empty_like(sd)
    scale = 0.125
    K().softmax_fwd(sd, p, None, B * H, H, Lq, Lk, ld, scale, spec)
    x = sd[..., :Lk].double().cpu() * scale
    pad = valid.lt(1)[:, None, None, :].expand(B, H, Lq, Lk)
    m = pad.clone()
    if Lq == Lk:
        m = m | pad.transpose(-1, -2) | torch.triu(torch.ones(Lq, Lk, dtype=torch.bool), 1)
    x = x.view(B, H, Lq, Lk).masked_fill(m, float("-inf"))
    ref = torch.nan_to_num(torch.softmax(x, -1)).view(B * H, Lq, Lk)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(p[..., :Lk].float().cpu(), ref) < tol
    assert (p.reshape(-1, ld)[:-1, Lk:] == 0).all()   # padding stored as zeros (all rows but the last)
    dpd = torch.randn(B * H, Lq, ld, generator=g).to(dev, dtype)
    ds = torch.empty_like(sd)
    K().softmax_bwd(p, dpd, ds, B * H, Lq, Lk, ld, scale)
    assert (ds.reshape(-1, ld)[:-1, Lk:] == 0).all()
    P = p[..., :Lk].double().cpu()
    G = dpd[..., :Lk].double().cpu()
    ref_ds = P * (G - (P * G).sum(-1, keepdim=True)) * scale
    assert relerr(ds[..., :Lk].float().cpu(), ref_ds) < tol * 2


@pytest.mark.parametrize("Lk", [129, 200, 249, 256])
@pytest.mark.parametrize("nbh,Lq", [(3, 7), (64, 601)])
def test_softmax_stream_unmasked(Lk, nbh, Lq):
    """The persistent streaming forward (bf16, no mask, no dropout output, 128 < Lk <= 256; softmax.hip
    softmax_fwd_stream_kernel): a row count that is not a multiple of 4 (the last row group), and 38 k rows — several
    row groups per wave, the prefetch ring — against torch; padding columns stored as zeros."""
    from asrx.kernels import MaskSpec
    g = torch.Generator().manual_seed(Lk + Lq)
    ld = (Lk + 7) // 8 * 8
    s = torch.randn(nbh, Lq, ld, generator=g) * 3
    sd = s.to(dev, torch.bfloat16)
    p = torch.full_like(sd, float("nan"))
    scale = 0.125
    K().softmax_fwd(sd, p, None, nbh, 1, Lq, Lk, ld, scale, MaskSpec())
    ref = torch.softmax(sd[..., :Lk].double().cpu() * scale, -1)
    assert relerr(p[..., :Lk].float().cpu(), ref) < 1e-2
    assert (p.reshape(-1, ld)[:-1, Lk:] == 0).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Lk", [24, 249])
@pytest.mark.parametrize("u", [0, 4])
def test_softmax_dropout(dtype, Lk, u, tuning):
    """Softmax with attention dropout p = 0.3 (layers.py:26): the forward's dropped copy pd = P * keep / (1 - p) and
    the backward dS = P * (G' - rowsum(P * G')) * scale with G' = dPd * keep / (1 - p), keep from rng_ref.attn_keep."""
    from asrx.kernels import MaskSpec
    from rng_ref import attn_keep
    tuning("softmax_u", u)
    B, H, Lq, p_drop, seed = 2, 3, min(Lk, 40), 0.3, 0x5EED1234ABCD
    g = torch.Generator().manual_seed(Lk + 1)
    ld = (Lk + 7) // 8 * 8
    s = torch.randn(B * H, Lq, ld, generator=g) * 3
    sd = s.to(dev, dtype)
    p = torch.empty_like(sd)
    pd = torch.empty_like(sd)
    scale = 0.125
    K().softmax_fwd(sd, p, pd, B * H, H, Lq, Lk, ld, scale, MaskSpec(), dropout_p=p_drop, seed=seed)
    keep = torch.from_numpy(attn_keep(seed, B * H, Lq, Lk, p_drop)).double()
    assert abs(float(keep.mean()) - (1 - p_drop)) < 0.05
    ref = torch.softmax(sd[..., :Lk].double().cpu() * scale, -1)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(p[..., :Lk].float().cpu(), ref) < tol
    P = p[..., :Lk].double().cpu()
    assert relerr(pd[..., :Lk].float().cpu(), P * keep / (1 - p_drop)) < tol
    assert torch.equal(pd[..., :Lk].cpu() == 0, keep == 0)   # exactly the dropped elements are zero
    dpd = torch.randn(B * H, Lq, ld, generator=g).to(dev, dtype)
    ds = torch.empty_like(sd)
    K().softmax_bwd(p, dpd, ds, B * H, Lq, Lk, ld, scale, dropout_p=p_drop, seed=seed)
    Gk = dpd[..., :Lk].double().cpu() * keep / (1 - p_drop)
    ref_ds = P * (Gk - (P * Gk).sum(-1, keepdim=True)) * scale
    assert relerr(ds[..., :Lk].float().cpu(), ref_ds) < tol * 2


# ------------------------------------------------------------------------------------------------ front-end

@pytest.mark.parametrize("T", [61, 1000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_frontend(dtype, T):
    B, F = 2, 80
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 1, F, T, generator=g)
    w1 = torch.randn(64, 1, 3, 3, generator=g) * 0.3
    b1 = torch.randn(64, generator=g) * 0.1
    w2 = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    F1, T1 = (F - 3) // 2 + 1, (T - 3) // 2 + 1
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    y1 = torch.empty(B, F1, T1, 64, device=dev, dtype=dtype)
    y1m = torch.empty(B, F1, T1, 8, device=dev, dtype=torch.uint8)
    K().conv1_fwd(x.to(dev), w1.reshape(64, 9).to(dev), b1.to(dev), y1, mask=y1m)
    bits = torch.stack([(y1m.cpu() >> i) & 1 for i in range(8)], -1).reshape(B, F1, T1, 64)
    assert torch.equal(bits.bool(), y1.float().cpu() > 0)
    ref1 = torch.relu(torch.nn.functional.conv2d(x.double(), w1.double(), b1.double(), stride=2))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(y1.float().cpu().permute(0, 3, 1, 2), ref1) < tol
    cols = torch.empty(B * T2 * F2, 576, device=dev, dtype=dtype)
    K().im2col_conv2(y1, cols)
    w2p = w2.permute(0, 2, 3, 1).reshape(64, 576).to(dev, dtype)
    y2 = torch.empty(B * T2 * F2, 64, device=dev, dtype=torch.float32)
    K().gemm(cols, w2p, y2, B * T2 * F2, 64, 576, lda=576, ldb=576, ldc=64)
    y1r = y1.float().cpu().permute(0, 3, 1, 2).double()
    ref2 = torch.nn.functional.conv2d(y1r, w2.to(dtype).double(), stride=2)        # (B,64,F2,T2)
    got = y2.cpu().view(B, T2, F2, 64).permute(0, 3, 2, 1)
    assert relerr(got, ref2) < tol
    if dtype == torch.bfloat16:   # implicit-GEMM conv2 (no im2col image), bias + ReLU fused
        b2 = torch.randn(64, generator=g) * 0.1
        y2i = torch.full((B * T2 * F2, 64), float("nan"), device=dev, dtype=dtype)
        K().conv2_fwd(y1, w2p, b2.to(dev), y2i)
        refi = torch.relu(ref2 + b2.double().view(1, 64, 1, 1))
        goti = y2i.float().cpu().view(B, T2, F2, 64).permute(0, 3, 2, 1)
        assert relerr(goti, refi) < tol
    # backward: dcols -> col2im (ReLU gate) and conv1 weight grads
    y1g = y1r.clone().requires_grad_(True)
    out2 = torch.nn.functional.conv2d(y1g, w2.to(dtype).double(), stride=2)
    gy = torch.randn(out2.shape, generator=g).double()
    out2.backward(gy)
    dy2 = gy.permute(0, 3, 2, 1).reshape(B * T2 * F2, 64).to(dev, dtype)
    dcols = torch.empty(B * T2 * F2, 576, device=dev, dtype=dtype)
    K().gemm(dy2, w2p, dcols, B * T2 * F2, 576, 64, lda=64, ldb=576, ldc=576, b_trans=True)
    if dtype == torch.bfloat16:   # conv2 weight/bias gradient with the im2col rows gathered from y1
        dw2 = torch.randn(64, 576, device=dev)
        db2 = torch.randn(64, device=dev)
        rw = dw2.double() + dy2.double().t() @ cols.double()
        rb = db2.double() + dy2.double().sum(0)
        K().conv2_wgrad(dy2, y1, dw2, db2)
        assert relerr(dw2, rw) < 1e-5
        assert relerr(db2, rb) < 1e-5
    dy1 = torch.empty(B, F1, T1, 64, device=dev)
    K().col2im_conv2(dcols, y1, dy1)
    ref_dy1 = (y1g.grad * (y1r > 0)).permute(0, 2, 3, 1)
    assert relerr(dy1.cpu(), ref_dy1) < tol * 2
    dw = torch.zeros(64, 9, device=dev)
    db = torch.zeros(64, device=dev)
    K().conv1_bwd_w(x.to(dev), dy1, dw, db)
    xr = x.double()
    w1r = w1.double().requires_grad_(True)
    b1r = b1.double().requires_grad_(True)
    pre = torch.nn.functional.conv2d(xr, w1r, b1r, stride=2)
    pre.backward(dy1.cpu().double().permute(0, 3, 1, 2))
    assert relerr(dw.cpu(), w1r.grad.reshape(64, 9)) < 1e-5
    assert relerr(db.cpu(), b1r.grad) < 1e-5
    # fused path (training): the same gradients straight from dcols, dy1 never materialised
    dw2 = torch.zeros(64, 9, device=dev)
    db2 = torch.zeros(64, device=dev)
    K().conv1_bwd_fused(dcols, y1, x.to(dev), dw2, db2)
    assert relerr(dw2.cpu(), w1r.grad.reshape(64, 9)) < 1e-4
    assert relerr(db2.cpu(), b1r.grad) < 1e-4
    if dtype == torch.bfloat16:   # implicit path: from dy2 itself, the column gradient never stored
        gyb = dy2.double().cpu().view(B, T2, F2, 64).permute(0, 3, 2, 1)
        y1g2 = y1r.clone().requires_grad_(True)
        torch.nn.functional.conv2d(y1g2, w2.to(dtype).double(), stride=2).backward(gyb)
        w1r2 = w1.double().requires_grad_(True)
        b1r2 = b1.double().requires_grad_(True)
        torch.nn.functional.conv2d(xr, w1r2, b1r2, stride=2).backward(y1g2.grad * (y1r > 0))
        dw3 = torch.zeros(64, 9, device=dev)
        db3 = torch.zeros(64, device=dev)
        K().conv_bwd_implicit(dy2, w2p, y1m, x.to(dev), dw3, db3)
        # (round 6: the conv1 weight gradient on bf16 MFMAs — bf16 dy1 and x, fp32 accumulation, the reference's
        #  autocast arithmetic: against the fp64 gradient of the bf16-rounded operands, and the exact one at bf16 level)
        w1r3 = w1.double().requires_grad_(True)
        b1r3 = b1.double().requires_grad_(True)
        gy1 = (y1g2.grad * (y1r > 0)).to(torch.bfloat16).double()
        torch.nn.functional.conv2d(xr.to(torch.bfloat16).double(), w1r3, b1r3, stride=2).backward(gy1)
        assert relerr(dw3.cpu(), w1r3.grad.reshape(64, 9)) < 1e-3
        assert relerr(db3.cpu(), b1r3.grad) < 1e-3
        assert relerr(dw3.cpu(), w1r2.grad.reshape(64, 9)) < 1e-2
        assert relerr(db3.cpu(), b1r2.grad) < 1e-2


# ------------------------------------------------------------------------------------------------ misc

@pytest.mark.parametrize("d,ntok", [(512, 4096), (80, 9000), (2048, 700), (12, 300)])
def test_embed_bwd_dropout_repeats(d, ntok):
    """Embedding gradient (nn.Embedding padding_idx backward of dropout(E[tok] + PE)) with dropout 0.1 and heavily
    repeated tokens (a few ids take most of the rows, more than one 4096-token chunk): against index_add of the
    masked, rescaled gradient rows, the keep mask from rng_ref (element index row * d + column)."""
    from rng_ref import elem_keep
    V, pad, p, seed = 250, 0, 0.1, 1234
    g = torch.Generator().manual_seed(9)
    tok = torch.randint(0, V, (ntok,), generator=g)
    tok[torch.rand(ntok, generator=g) < 0.3] = 1      # a very frequent id (BOS / EOS-like)
    tok[torch.rand(ntok, generator=g) < 0.2] = pad
    dout = torch.randn(ntok, d, generator=g)
    keep = torch.from_numpy(elem_keep(seed, ntok * d, p).reshape(ntok, d).astype(np.float32))
    ref = torch.zeros(V, d, dtype=torch.float64)
    ref.index_add_(0, tok, (dout * keep / (1 - p)).double())
    ref[pad] = 0
    dE = torch.zeros(V, d, device=dev)
    K().embed_bwd(tok.to(dev), dout.to(dev), dE, 64, pad_id=pad, dropout_p=p, seed=seed)
    assert relerr(dE.cpu().double(), ref) < 1e-6


def test_embedding_and_ce_and_adam():
    V, d, B, L = 250, 128, 4, 16
    g = torch.Generator().manual_seed(6)
    E = torch.randn(V, d, generator=g)
    pe = torch.randn(32, d, generator=g)
    tok = torch.randint(0, V, (B, L), generator=g)
    tok[0, -3:] = 4
    out = torch.empty(B * L, d, device=dev)
    K().embed_fwd(tok.to(dev), E.to(dev), pe.to(dev), out, L)
    ref = E[tok.reshape(-1)] + pe[torch.arange(B * L) % L]
    assert relerr(out.cpu(), ref) < 1e-6
    dout = torch.randn(B * L, d, generator=g)
    dE = torch.zeros(V, d, device=dev)
    K().embed_bwd(tok.to(dev), dout.to(dev), dE, L, pad_id=4)
    Er = E.clone().requires_grad_(True)
    torch.nn.functional.embedding(tok.reshape(-1), Er, padding_idx=4).backward(dout)
    assert relerr(dE.cpu(), Er.grad) < 1e-6
    # cross entropy with padded logits
    rows, Vp = 37, 256
    logits = torch.randn(rows, Vp, generator=g) * 3
    tgt = torch.randint(0, V, (rows,), generator=g)
    tgt[5] = -100
    loss, dl, am = K().cross_entropy(logits.to(dev), V, tgt.to(dev), want_argmax=True)
    lr = logits[:, :V].double().requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(lr, tgt)
    lref.backward()
    lref = lref.detach()
    assert abs(float(loss) - float(lref)) < 1e-5 * abs(float(lref))
    assert relerr(dl[:, :V].float().cpu(), lr.grad) < 1e-2
    assert torch.all(dl[:, V:] == 0)
    assert torch.equal(am.cpu(), logits[:, :V].argmax(-1))
    # adam vs torch.optim.Adam
    n = 1003
    p0 = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pt], lr=1e-3, betas=(0.9, 0.98), eps=1e-9, weight_decay=0.01)
    pd, md, vd = p0.clone().to(dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in (1, 2, 3):
        pt.grad = gr * step
        opt.step()
        K().adam(pd, (gr * step).to(dev), md, vd, pb, 1e-3, 0.9, 0.98, 1e-9, 0.01, step, decoupled=True)
    assert relerr(pd.cpu(), pt.detach()) < 1e-6
    assert relerr(pb.float().cpu(), pt.detach()) < 1e-2


@pytest.mark.parametrize("world,chunk", [(1, 7), (2, 1000), (8, 12345), (3, 0)])
def test_sum_chunks_bf16(world, chunk):
    """bf16-wire gradient exchange (asrx.dist wire="bf16"): the W peers' bf16 chunks summed in fp32, rounded once."""
    g = torch.Generator(device=dev).manual_seed(world * 7 + chunk)
    recv = bf(torch.randn(world * chunk, device=dev, generator=g) * 3)
    out = torch.empty(chunk, device=dev, dtype=torch.bfloat16)
    K().sum_chunks_bf16(recv, world, chunk, out)
    want = recv.view(world, chunk).float().sum(0).to(torch.bfloat16) if chunk else out
    assert torch.equal(out, want)


def test_zero_spans_and_step_tokens():
    """asrx_zero_spans (the step's gradient zeroing: ragged, unaligned and adjacent spans, nothing outside them
    touched) and asrx_step_tokens (decoder input, targets and validity mask of train.py:22-24,32 / model.py:108-115)
    against torch."""
    g = torch.Generator(device=dev).manual_seed(3)
    buf = torch.randn(100003, device=dev, generator=g)
    ref = buf.clone()
    spans = [(0, 5), (5, 64), (70, 71), (77, 4099), (5000, 5003), (9001, 70001), (99999, 100003)]
    for a, b in spans:
        ref[a:b] = 0
    K().zero_spans(buf, torch.tensor(spans, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    B, L1 = 5, 17
    text = torch.randint(0, 250, (B, L1), device=dev, generator=g)
    inp = torch.randint(0, 250, (B, L1), device=dev, generator=g)
    mask = (torch.rand(B, L1, device=dev, generator=g) > 0.3).float()
    dec_in, tgt, valid = K().step_tokens(text, inp, mask)
    torch.cuda.synchronize()
    assert torch.equal(dec_in.view(B, L1 - 1), inp[:, :-1])
    assert torch.equal(tgt, text[:, 1:].reshape(-1))
    assert torch.equal(valid, (mask[:, :-1] >= 1).to(torch.uint8))
