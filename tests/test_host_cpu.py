"""Host-side checks that need no GPU: the C-ABI library loads and exports every declared symbol, the
drop-in modules reproduce the reference state_dict schema exactly, and the storage re-layouts
(fused per-head projections, permuted _lin_in columns, channels-last conv2, padded classifier, flat
parameter store) are lossless."""
import json
import os
import re

import pytest
import torch

from oracle.ref_model import CONFIGS, det_params

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "asrx.h")).read()
    return sorted(set(re.findall(r"\b(?:int|int64_t)\s+(asrx_\w+)\s*\(", src)))


# entry points with a non-int result, bound separately in asrx._lib.lib()
_NON_INT = {"asrx_attn_dropmask_words", "asrx_attn_dq_acc_elems"}


def test_library_exports_every_declared_symbol():
    import asrx
    from asrx._lib import SIGNATURES
    lib = asrx.native()
    syms = _declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in SIGNATURES or s in _NON_INT, s
    assert set(SIGNATURES) | _NON_INT == set(syms)
    assert lib.asrx_version() >= 1


@pytest.mark.parametrize("B,H,Lq,Lk", [(64, 8, 249, 249), (16, 8, 999, 999), (2, 8, 64, 300), (1, 1, 1, 257),
                                       (3, 4, 33, 256)])
def test_dropmask_size_rule(B, H, Lq, Lk):
    """The header's dropmask size rule (asrx_attn_dropmask_words): key-major [B*H][ceil(Lq/32)][Lk] words, then
    query-major [B*H][Lq][qmaj_stride(Lk)] with the stride rounded up to a multiple of 4 past 256 keys."""
    import asrx
    from asrx.kernels import qmaj_stride
    lib = asrx.native()
    nkw = (Lk + 31) // 32
    stride = nkw if Lk <= 256 else (nkw + 3) // 4 * 4
    assert qmaj_stride(Lk) == stride
    assert lib.asrx_attn_dropmask_words(B, H, Lq, Lk) == B * H * (((Lq + 31) // 32) * Lk + Lq * stride)
    assert lib.asrx_attn_dropmask_words(0, H, Lq, Lk) == -1
    # dq_acc (version 3): one [B*Lq*H*dh] fp32 slab per 128 keys past 128 keys, none below
    assert lib.asrx_version() >= 3
    assert lib.asrx_attn_dq_acc_elems(B, H, Lq, Lk, 64) == (0 if Lk <= 128 else (Lk + 127) // 128 * B * Lq * H * 64)
    assert lib.asrx_attn_dq_acc_elems(B, H, Lq, Lk, 48) == -1


def test_abi_rejects_bad_arguments_without_gpu():
    """Argument validation happens before any launch: a NULL descriptor must return ASRX_ERR_ARG."""
    import asrx
    lib = asrx.native()
    assert lib.asrx_gemm(None, None) == -1
    assert lib.asrx_attention_fwd(None, None) == -1
    assert lib.asrx_cast(0, None, 0, None, 10, None) == -1


def test_ctypes_struct_sizes_match_the_library():
    """Every descriptor struct mirrored in the ctypes binding has the size the library was compiled with
    (asrx_struct_sizes): a stale mirror would make the library read past the caller's struct."""
    import ctypes
    import asrx
    from asrx._lib import AdamDesc, AttnDesc, GemmDesc, GemmGroupDev, RowsumGroup
    lib = asrx.native()
    out = (ctypes.c_int64 * 5)()
    assert lib.asrx_struct_sizes(out, 5) == 5
    assert list(out) == [ctypes.sizeof(GemmDesc), ctypes.sizeof(AttnDesc), ctypes.sizeof(GemmGroupDev),
                         ctypes.sizeof(RowsumGroup), ctypes.sizeof(AdamDesc)]
    assert ctypes.sizeof(GemmGroupDev) == 64


def test_abi_upload_and_seed_offset_validate_arguments_without_gpu():
    import asrx
    lib = asrx.native()
    assert lib.asrx_upload(None, None, 16, None) == -1
    assert lib.asrx_upload(4096, None, 6, None) == -1      # nbytes not a multiple of 4


def _build(name, **kw):
    import asrx
    cfg = CONFIGS[name]["cfg"]
    return asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                            cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, **kw), cfg


@pytest.mark.parametrize("name", ["micro", "c1", "c3"])
def test_state_dict_schema_matches_reference(golden_dir, name):
    ref = json.load(open(os.path.join(golden_dir, "ref_state_dict_schema.json")))
    m, cfg = _build(name)
    sd = m.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == ref[name]
    # parameter count: ours pads the classifier rows to a multiple of 64 and nothing else
    pad = (m.decoder._classifier.Vp - cfg.vocab_size) * cfg.d_model
    assert sum(p.numel() for p in m.parameters()) == ref[name + "_nparams"] + pad


def test_reference_weights_round_trip_exactly():
    m, cfg = _build("c1")
    P = det_params(cfg, 3)
    sd = m.state_dict()
    sd.update(P)
    m.load_state_dict(sd)
    out = m.state_dict()
    for k, v in P.items():
        assert torch.equal(out[k], v), k
    # internal layouts
    d, H = cfg.d_model, cfg.n_heads
    dh = d // H
    mha = m.encoder._layers[1]._attention
    for i in range(H):
        assert torch.equal(mha.wqkv[i * dh:(i + 1) * dh], P[f"encoder._layers.1._attention._heads.{i}._q.weight"])
        assert torch.equal(mha.wqkv[d + i * dh:d + (i + 1) * dh],
                           P[f"encoder._layers.1._attention._heads.{i}._k.weight"])
        assert torch.equal(mha.bqkv[2 * d + i * dh:2 * d + (i + 1) * dh],
                           P[f"encoder._layers.1._attention._heads.{i}._v.bias"])
    ca = m.decoder._layers[0]._cross_attention
    assert torch.equal(ca.wkv[:d], torch.cat([P[f"decoder._layers.0._cross_attention._heads.{i}._k.weight"]
                                              for i in range(H)]))
    W = P["encoder._lin_in.weight"]              # (d, c*F2 + f)
    F2 = W.shape[1] // 64
    phys = m.encoder._lin_in.weight.detach()     # (d, f*64 + c)
    assert torch.equal(phys.view(d, F2, 64)[:, 5, 7], W.view(d, 64, F2)[:, 7, 5])
    w2 = m.input_layer[2].weight
    assert w2.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(w2, P["input_layer.2.weight"])
    assert torch.all(m.decoder._classifier.weight[cfg.vocab_size:] == 0)


def test_flat_store_layout_on_cpu():
    from asrx.functions import param_order
    from asrx.params import ALIGN, FlatParams
    m, cfg = _build("micro")
    before = {k: v.clone() for k, v in m.state_dict().items()}
    st = FlatParams(param_order(m), "cpu")
    after = m.state_dict()
    for k in before:
        assert torch.equal(before[k], after[k]), k
    for p in m.parameters():
        assert p.data.data_ptr() == st.flat.data_ptr() + 4 * st.offset(p)
        assert st.offset(p) % ALIGN == 0
        assert p.grad is not None and p.grad.data_ptr() == st.grad.data_ptr() + 4 * st.offset(p)
    # the decoder's cross-attention K/V projections form one contiguous [n_dec*2d, d] block
    dec = m.decoder
    n, d = len(dec._layers), cfg.d_model
    span = st.span(dec._layers[0]._cross_attention.wkv, n, st.flat)
    assert span is not None and span.numel() == n * 2 * d * d
    # LayerNorm gamma/beta adjacent (one fused dgamma|dbeta reduction)
    ln = m.encoder._layers[0]._norm1
    assert st.offset(ln.bias) == st.offset(ln.weight) + d
    # conv2 weight keeps its channels-last physical layout inside the store
    assert m.input_layer[2].weight.is_contiguous(memory_format=torch.channels_last)


def test_modules_refuse_cpu_execution():
    """No CPU fallback: running the drop-in model without a GPU raises instead of silently computing."""
    m, cfg = _build("micro")
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 1, 80, 60), torch.ones(1, 8, dtype=torch.long), torch.ones(1, 8))


def test_gemm_kernel_plan_names_without_gpu():
    """The kernel-selection policy is host logic: query it through the C-ABI with fake (aligned) pointers."""
    from asrx._lib import BF16, F32, GemmDesc
    from asrx.kernels import kernel_name

    def desc(m, n, k, at=0, bt=0, bias=False, c_dtype=BF16, in_dtype=BF16):
        d = GemmDesc()
        d.m, d.n, d.k, d.in_dtype = m, n, k, in_dtype
        d.a, d.lda, d.a_trans = 1 << 20, (m if at else k), at
        d.b, d.ldb, d.b_trans = 2 << 20, (n if bt else k), bt
        d.c, d.ldc, d.c_dtype = 3 << 20, n, c_dtype
        d.alpha, d.batch, d.batch_inner, d.splitk = 1.0, 1, 1, 1
        if bias:
            d.bias = 4 << 20
        return d

    # wide outputs (>= 400 256x256 tiles) take p4; the Q/K/V projection forward (bias) the ws kernel, encoder and
    # decoder (round 4's persistent ws variants, codes 9 and 11, were removed in round 5: they plan as auto)
    assert kernel_name(desc(15936, 1536, 512, bias=True)) == "gemm_bf16_ws_kernel<false, 1, 256>"
    assert kernel_name(desc(4096, 1536, 512, bias=True)) == "gemm_bf16_ws_kernel<false, 1, 256>"
    assert kernel_name(desc(15936, 1536, 512)) == "gemm_bf16_p3_kernel<false, false, 0>"
    forced = desc(15936, 1536, 512, bias=True)
    for code in (9, 11):
        forced.kernel = code
        assert kernel_name(forced) == "gemm_bf16_ws_kernel<false, 1, 256>"
    assert kernel_name(desc(15936, 2048, 512, bt=1)) == "gemm_bf16_p4_kernel<false, true, 0>"
    ffn1 = desc(15936, 2048, 512, bias=True)
    ffn1.relu = 1
    # (bias + ReLU on p4 runs as the dropout instantiation with threshold 0: the plain one spills, gemm.hip)
    assert kernel_name(ffn1) == "gemm_bf16_p4_kernel<false, false, 7>"
    ragged = desc(1000, 4160, 256, bias=True)   # N % 128 != 0: a forced ws-family code plans as auto
    ragged.kernel = 8
    assert kernel_name(ragged) == kernel_name(desc(1000, 4160, 256, bias=True))
    assert kernel_name(desc(15936, 12288, 512, bias=True)) == "gemm_bf16_p4_kernel<false, false, 1>"
    forced.kernel = 6                 # p4 forced: the 256x256 ring
    assert kernel_name(forced) == "gemm_bf16_p4_kernel<false, false, 1>"
    # the plain 512-wide data gradients with K >= 1536 take the warp-specialised ws kernel, shorter ones stay on p3
    assert kernel_name(desc(15936, 512, 2048, bt=1)) == "gemm_bf16_ws_kernel<true, 0, 256>"
    assert kernel_name(desc(15936, 512, 1536, bt=1)) == "gemm_bf16_ws_kernel<true, 0, 256>"
    assert kernel_name(desc(15936, 512, 512, bt=1)) == "gemm_bf16_ws_kernel<true, 0, 256>"
    # the decoder's 4096-row ones on ws with 64 x 128 tiles (one per CU)
    assert kernel_name(desc(4096, 512, 2048, bt=1)) == "gemm_bf16_ws_kernel<true, 0, 64>"
    assert kernel_name(desc(4096, 512, 512, bt=1)) == "gemm_bf16_ws_kernel<true, 0, 64>"
    assert kernel_name(desc(1024, 512, 2048, bt=1)).startswith("gemm_bf16_ring_kernel")
    assert kernel_name(desc(15936, 512, 512, bias=True)) == "gemm_bf16_ws_kernel<false, 1, 256>"
    # the FFN2 forward (bias + fp32 residual, fp32 out, K = 2048) on ws, the decoder's 4096-row one on 64-row tiles
    ff2 = desc(15936, 512, 2048, bias=True, c_dtype=F32)
    ff2.resid, ff2.ld_resid, ff2.resid_dtype = 5 << 20, 512, F32
    assert kernel_name(ff2) == "gemm_bf16_ws_kernel<false, 81, 256>"
    ff2.m = 4096
    assert kernel_name(ff2) == "gemm_bf16_ws_kernel<false, 81, 64>"
    wg = desc(2048, 512, 15936, at=1, bt=1, c_dtype=F32)
    wg.tile = 128                     # as kernels.wgrad_plan sets it
    assert kernel_name(wg) == "gemm_bf16_kernel<128, 128, true, true, true>"
    assert kernel_name(desc(64, 64, 64, in_dtype=F32, c_dtype=F32)) == "gemm_f32_kernel<false, false>"
    d7 = desc(15936, 512, 2048, bt=1)
    d7.kernel = 7                     # no library family exists any more: the retired code plans automatically
    assert kernel_name(d7) == "gemm_bf16_ws_kernel<true, 0, 256>"
    d7.kernel = 10                    # ws on 64 x 128 tiles, forced
    assert kernel_name(d7) == "gemm_bf16_ws_kernel<true, 0, 64>"
    forced = desc(15936, 1536, 512)
    forced.kernel = 3  # noqa                 # asrx_gemm_desc.kernel: register-staged family
    assert kernel_name(forced).startswith("gemm_bf16_kernel<128, 128, false, false, true>")


def test_rng_restatement_statistics():
    """The numpy RNG restatement (test oracle of the dropout masks) keeps 1-p of the elements, pairs halves of
    one hash, and attention pairs run along queries."""
    import numpy as np
    from rng_ref import attn_keep, elem_keep, rng_hash, threshold
    assert threshold(0.1) == 6554 and threshold(0) == 0 and threshold(1.0) == 65536
    k = elem_keep(7, 1 << 20, 0.1)
    assert abs(k.mean() - 0.9) < 0.002
    h = rng_hash(7, np.arange(4, dtype=np.uint64))
    assert len(set(h.tolist())) == 4
    a = attn_keep(7, 3, 9, 13, 0.25)
    assert a.shape == (3, 9, 13) and abs(a.mean() - 0.75) < 0.1
    assert not elem_keep(7, 1000, 1.0).any() and elem_keep(7, 1000, 0.0).all()


def test_release_spans_are_exact():
    """The gradient ranges released to the all-reduce cover exactly the given params (no neighbours)."""
    from asrx.functions import _spans, param_order
    from asrx.params import FlatParams
    m, cfg = _build("c1")
    st = FlatParams(param_order(m), "cpu")

    class C:
        store = st
    enc = m.encoder
    params = [p for p in enc._layers[1].parameters()] + list(enc._norm_out.parameters())
    spans = _spans(C, params)
    covered = sum(b - a for a, b in spans)
    mine = {id(p) for p in params}
    for p in st.params:   # no other parameter overlaps a span
        o = st.offset(p)
        inside = any(a <= o < b for a, b in spans)
        assert inside == (id(p) in mine), p.shape
    assert covered >= sum(p.numel() for p in params)
    assert len(_spans(C, list(m.decoder.parameters()))) == 1


def _c3_wgrad_shapes():
    enc, dec, d, ff = 15936, 4096, 512, 2048
    shapes = []
    for _ in range(12):
        shapes += [(3 * d, d, enc), (d, d, enc), (ff, d, enc), (d, ff, enc)]
    for _ in range(12):
        shapes += [(3 * d, d, dec), (d, d, dec), (d, d, dec), (d, d, dec), (ff, d, dec), (d, ff, dec)]
    return shapes + [(12 * 2 * d, d, enc), (d, 19 * 64, enc), (256, d, dec)]


@pytest.mark.parametrize("pack", [False, True])
def test_xcd_plan_covers_every_tile_once(pack):
    """The grouped weight-gradient workgroup -> tile map (kernels.xcd_plan) at the c3 step's shapes: every tile of
    every group exactly once, tiles of a group contiguous in the tile numbering, and (pack) each group's tiles on
    one XCD, in rounds of at most 32 per XCD that never split a group of <= 32 tiles."""
    import numpy as np
    from asrx import kernels
    shapes = _c3_wgrad_shapes()
    group_order, nts, block_tile, tmap = kernels.xcd_plan(shapes, tile=256, nxcd=8, pack=pack)
    assert sorted(group_order) == list(range(len(shapes)))
    total = sum(nts)
    used = block_tile[block_tile != 0xFFFF].astype(np.int64)
    assert sorted(used.tolist()) == list(range(total))
    assert len(tmap) == total
    starts = np.cumsum([0] + [nts[i] for i in group_order])
    for slot, i in enumerate(group_order):
        assert (tmap[starts[slot]:starts[slot + 1]] == slot).all()
    for x in range(8):
        col = block_tile[x::8]
        col = col[col != 0xFFFF].astype(np.int64)
        groups = tmap[col]
        for slot in set(groups.tolist()):
            pos = np.nonzero(groups == slot)[0]
            assert pos[-1] - pos[0] + 1 == len(pos)          # a group's tiles are consecutive on its XCD
        if pack:
            for slot in set(groups.tolist()):
                n = nts[group_order[slot]]
                pos = np.nonzero(groups == slot)[0]
                if n <= 32 and len(pos) == n:
                    assert len(pos) <= 32
    # each group on exactly one XCD (the packed plan may split a group of > 32 tiles over XCDs)
    where = {}
    for b, t in enumerate(block_tile.tolist()):
        if t != 0xFFFF:
            where.setdefault(int(tmap[t]), set()).add(b % 8)
    for slot, xs in where.items():
        if not pack or nts[group_order[slot]] <= 32:
            assert len(xs) == 1


def test_early_adam_spans_cover_the_buffer_once():
    """Trainer._reduce_and_adam's split of the flat buffer: the released ranges shrunk to 16-B aligned spans plus
    their complement cover every element exactly once, and every span starts 4-element aligned."""
    from asrx.train import _aligned_spans, _complement
    import random
    rng = random.Random(0)
    for _ in range(200):
        n = rng.randrange(1, 5000)
        spans = []
        for _ in range(rng.randrange(0, 6)):
            a = rng.randrange(0, n)
            spans.append((a, rng.randrange(a, n + 1)))
        early = _aligned_spans(spans, n)
        late = _complement(early, n)
        cover = [0] * n
        for a, b in early + late:
            assert a % 4 == 0
            for i in range(a, b):
                cover[i] += 1
        assert cover == [1] * n
        released = set(i for a, b in spans for i in range(a, b))
        assert all(i in released for a, b in early for i in range(a, b))


def _build_new(name):
    import asrx.new
    from oracle.ref_model_new import NEW_CONFIGS
    c = NEW_CONFIGS[name]
    m = asrx.new.Transformer(c.vocab_size, c.n_mels, c.enc_seq_len, c.dec_seq_len, c.hidden_dim, c.n_enc, c.n_dec,
                             c.n_heads, c.ff_dim, "cpu", dropout=c.dropout, sr=c.sr, n_fft=c.n_fft, padding_idx=c.pad_id,
                             eos_token=c.eos_id, bos_token=c.bos_id)
    return m, c


@pytest.mark.parametrize("name", ["new_micro", "new_small"])
def test_new_state_dict_schema_matches_reference(golden_dir, name):
    """asrx.new.Transformer (the post-LN family, modules/Transformer/new/) has the reference's state_dict keys,
    order and shapes (tests/golden/make_golden_new.py records them from the reference), and its fused per-head
    q / k / v storage round-trips a reference state_dict losslessly."""
    from oracle.ref_model_new import det_params
    ref = json.load(open(os.path.join(golden_dir, "ref_new_state_dict_schema.json")))
    m, c = _build_new(name)
    sd = m.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == ref[name]
    assert sum(p.numel() for p in m.parameters()) == ref[name + "_nparams"]
    P = det_params(c, 0)
    sd.update(P)
    m.load_state_dict(sd)
    back = m.state_dict()
    for k, v in P.items():
        assert torch.equal(back[k], v), k


def test_fused_adam_residual_pieces():
    """The ranges the span-table AdamW steps after a fused weight-gradient launch: the complement of the covered
    parameters, cut into bounded pieces, every element of the buffer stepped exactly once over cover + pieces."""
    from asrx.train import residual_pieces
    n = 10_000
    cover = [(64, 256), (1024, 512), (320, 64), (9_984, 16)]
    pieces = residual_pieces(n, cover, piece=1000)
    assert all(b - a <= 1000 and a % 4 == 0 and b % 4 == 0 for a, b in pieces)
    hits = [0] * n
    for o, k in cover:
        for i in range(o, o + k):
            hits[i] += 1
    for a, b in pieces:
        for i in range(a, b):
            hits[i] += 1
    assert hits == [1] * n
    assert residual_pieces(128, [(0, 128)]) == []


def test_new_over_length_inputs_raise():
    """asrx.new: frames past the encoder's positional table, or tokens past the decoder's, raise ValueError before
    any device work (the reference's `x + pe[:, :T]` fails to broadcast there; embed_fwd would read past the table)."""
    m, c = _build_new("new_micro")
    T = m.encoder.pe.pe.shape[1] + 1
    with pytest.raises(ValueError):
        m.encoder(torch.zeros(1, 1, c.n_mels, T), torch.tensor([T]))
    L = m.decoder.pe.pe.shape[1] + 1
    with pytest.raises(ValueError):
        m.decoder(torch.zeros(1, L, dtype=torch.int64), torch.zeros(1, 4, c.n_mels), torch.tensor([4]))


def test_device_code_has_no_sgpr_hazard_before_vector_memory():
    """No VALU write of an SGPR within 5 wait states of a buffer / global instruction reading it, no VALU
    overwrite of a 16-B store's data right after it, no LDS-DMA right after an M0 write and no load's destination
    touched before a wait that proves it landed, in any built kernel (tools/asm_hazards.py: the compiler pads
    neither around inline asm; round 5's loader-wave AdamW experiment faulted on the one, corrupted moments by the
    other)."""
    import glob
    import shutil
    import sys
    objs = sorted(glob.glob(os.path.join(REPO, "asr-transformer_amd", "asrx", "lib", "*.o")))
    if not objs or not shutil.which("objcopy") or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("built objects / ROCm binutils not present")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    try:
        import asm_hazards
    finally:
        sys.path.pop(0)
    bad = []
    for o in objs:
        dis = asm_hazards.disassemble(o)
        bad += [(os.path.basename(o), h) for h in asm_hazards.scan_text(dis) + asm_hazards.scan_loads(dis)]
    assert not bad, bad[:5]
    # the scanner itself sees the faulting pattern
    assert asm_hazards.scan_text("v_readlane_b32 s83, v253, 57\nbuffer_store_dwordx2 v[2:3], v6, s[80:83], 0 offen")
    assert not asm_hazards.scan_text(
        "v_readlane_b32 s83, v253, 57\ns_nop 4\nbuffer_store_dwordx2 v[2:3], v6, s[80:83], 0 offen")
    assert asm_hazards.scan_text("buffer_store_dwordx4 v[22:25], v39, s[76:79], 0 offen\nv_cndmask_b32_e64 v22, 0, 1, s[80:81]")
    assert not asm_hazards.scan_text(
        "buffer_store_dwordx4 v[22:25], v39, s[76:79], 0 offen\ns_nop 1\nv_cndmask_b32_e64 v22, 0, 1, s[80:81]")
    assert asm_hazards.scan_text("s_mov_b32 m0, s4\nbuffer_load_dwordx4 v2, s[28:31], 0 offen lds")
    assert not asm_hazards.scan_text("s_mov_b32 m0, s4\ns_nop 0\nbuffer_load_dwordx4 v2, s[28:31], 0 offen lds")
    # a load's destination read before a wait that proves it landed (an inline-asm load hipcc does not count)
    two = "global_load_dwordx4 v[2:5], v[0:1], off\nglobal_load_dwordx4 v[6:9], v[0:1], off\ns_waitcnt vmcnt(1)\n"
    assert not asm_hazards.scan_loads(two + "v_mov_b32 v10, v2")
    assert asm_hazards.scan_loads(two + "v_mov_b32 v10, v6")
