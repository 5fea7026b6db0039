"""Tensor-level wrappers around the C-ABI (include/asrx.h). All calls are asynchronous on torch's current
HIP stream; every call goes to the native library (no CPU / PyTorch fallback)."""
import ctypes
import os
import math

import torch

from ._lib import MAX_ROWSUM_GROUPS, AttnDesc, BF16, BITS, F32, GemmDesc, RowsumGroup, call

_U64 = (1 << 64) - 1


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_dev = torch._C._cuda_getDevice


def stream():
    """Raw handle of torch's current HIP stream on the current device (honours `with torch.cuda.stream(...)`
    and graph capture); the cheap C accessors, not torch.cuda.current_stream() (≈9 µs of Python per call)."""
    return _raw_stream(_cur_dev())


def code(t):
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    raise TypeError(f"asrx: unsupported dtype {t.dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def _cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("asrx: tensors must live on the GPU (no CPU fallback)")


# ------------------------------------------------------------------------------------------- GEMM

def auto_splitk(m, n, k, batch=1, tile=64):
    """Split the reduction when the output grid alone cannot fill the 256 CUs (dW GEMMs: K = B*T)."""
    if batch != 1:
        return 1
    tiles = math.ceil(m / tile) * math.ceil(n / tile)
    if tiles >= 256 or k < 1024:
        return 1
    s = min(math.ceil(512 / tiles), max(1, k // 512), 256)
    return max(1, s)


class KernelProbe:
    """Brackets GEMM launches with HIP events on the launching stream (bench.py roofline), keyed by the kernel
    instantiation asrx_gemm_kernel_name reports — the same name rocprofv3 lists, so the live average agrees
    with the profiler's.  target=None records every GEMM (to find the dominant one); otherwise only launches
    of `target` are timed."""

    def __init__(self, target=None, log=None):
        self.target = target
        self.events = {}            # name -> [(start, end)]
        self.flops = {}             # name -> algorithmic FLOPs
        self.alg_bytes = {}         # name -> algorithmic HBM bytes of one launch (where the launch site states them)
        self.active = False
        self.log = log              # optional list: (kernel name, m, n, k, batch, splitk) of every GEMM launch

    def record(self, name):
        return self.active and (self.target is None or name == self.target)

    def durations_ms(self, name):
        return [s.elapsed_time(e) for s, e in self.events.get(name, [])]

    def dominant(self):
        tot = {n: sum(self.durations_ms(n)) for n in self.events}
        return max(tot, key=tot.get) if tot else None


# the _Segments of a training step being captured as HIP graphs (asrx.train.Trainer), else None
CAPTURE = None


def timed_launch(name, flops, launch):
    """Run launch(); if the active probe times `name`, bracket it with HIP events on the launching stream — or,
    while a step is being captured, give it a graph segment of its own that the replay brackets with events."""
    probe = PROBE
    if probe is None or not probe.record(name):
        launch()
        return
    if CAPTURE is not None:          # every replay of this segment adds `flops` (asrx.train._Segments.replay)
        CAPTURE.split((name, flops))
        launch()
        CAPTURE.split(None)
        return
    probe.flops[name] = probe.flops.get(name, 0) + flops
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    launch()
    s1.record()
    probe.events.setdefault(name, []).append((s0, s1))


def kernel_name(d):
    buf = ctypes.create_string_buffer(128)
    call("asrx_gemm_kernel_name", ctypes.byref(d), buf, 128)
    return buf.value.decode()


PROBE = None

# asrx_gemm_desc.kernel: forced kernel family (0 = auto).  ASRX_GEMM_KERNEL picks a process-wide default (A/B).
KERNEL_CODES = {"auto": 0, "p3": 1, "reg": 3, "ring": 4, "ring128": 5, "p4": 6, "ws": 8, "ws64": 10}
GEMM_KERNEL = KERNEL_CODES.get(os.environ.get("ASRX_GEMM_KERNEL", "auto"), 0)


def choose_tile(m, n, batch, splitk):
    t128 = math.ceil(m / 128) * math.ceil(n / 128) * batch * splitk
    return 128 if t128 >= 400 else 64


def gemm(a, b, c, m, n, k, *, lda, ldb, ldc, a_trans=False, b_trans=False, alpha=1.0, beta=0.0, bias=None,
         rowadd=None, rowadd_mod=1, ld_rowadd=0, relu=False, dropout_p=0.0, seed=0, gate=None, ld_gate=0,
         resid=None, ld_resid=0, batch=1, batch_inner=1, sa=(0, 0), sb=(0, 0), sc=(0, 0), splitk=1, tile=0,
         rowsum=None, gate_bits=False, mask_out=None, ld_mask=0, kernel=None):
    """C = epi(alpha * op(A) op(B)^T) — see asrx_gemm in include/asrx.h.  kernel: forced kernel family
    (KERNEL_CODES name or asrx_gemm_desc.kernel code; tests / A-B), default GEMM_KERNEL.  rowsum (fp32 [m], a_trans only):
    += row sums of A (fused bias gradient).  gate_bits: gate is an int32 bit mask [m][ld_gate words]
    (ASRX_BITS).  mask_out (int32 [m][ld_mask words]) receives the bits C > 0 (see asrx_gemm_desc)."""
    _cuda(a, b, c)
    if a.dtype != b.dtype:
        raise TypeError("asrx.gemm: A and B must share a dtype")
    if splitk == "auto":
        splitk = auto_splitk(m, n, k, batch)
    if tile == 0 and a.dtype == torch.bfloat16:
        tile = choose_tile(m, n, batch, splitk)
    ws = None
    wsp, wse, rwsp = None, 0, None
    if splitk > 1:
        ws = torch.empty(splitk * m * n, device=c.device, dtype=torch.float32)
        wsp, wse = ws.data_ptr(), ws.numel()
    else:
        splitk = 1
    if rowsum is not None:
        _cuda(rowsum)
        if splitk > 1:
            rws = torch.empty(splitk * m, device=c.device, dtype=torch.float32)
            rwsp = rws.data_ptr()
    # one positional constructor call (field order of GemmDesc / asrx_gemm_desc): far cheaper than ~30 setattrs
    d = GemmDesc(m, n, k, code(a),
                 a.data_ptr(), lda, int(a_trans), b.data_ptr(), ldb, int(b_trans), c.data_ptr(), ldc, code(c),
                 batch, batch_inner, sa[0], sa[1], sb[0], sb[1], sc[0], sc[1], alpha, beta,
                 None if bias is None else bias.data_ptr(),
                 None if rowadd is None else rowadd.data_ptr(), ld_rowadd if rowadd is not None else 0,
                 rowadd_mod if rowadd is not None else 0, int(relu), dropout_p, seed & _U64,
                 None if gate is None else gate.data_ptr(), ld_gate if gate is not None else 0,
                 (BITS if gate_bits else code(gate)) if gate is not None else 0,
                 None if resid is None else resid.data_ptr(), ld_resid if resid is not None else 0,
                 code(resid) if resid is not None else 0,
                 splitk, wsp, wse, tile, None if rowsum is None else rowsum.data_ptr(), rwsp,
                 None if mask_out is None else mask_out.data_ptr(), ld_mask if mask_out is not None else 0,
                 KERNEL_CODES.get(kernel, kernel) if kernel is not None else GEMM_KERNEL)
    probe = PROBE
    if probe is not None and probe.active:
        name = kernel_name(d)
        if probe.log is not None:
            probe.log.append((name, m, n, k, batch, splitk))
        timed_launch(name, 2 * m * n * k * batch, lambda: call("asrx_gemm", ctypes.byref(d), stream()))
        return ws
    call("asrx_gemm", ctypes.byref(d), stream())
    return ws


def linear(x, w, out, *, bias=None, **kw):
    """out[M,N] = x[M,K] . w[N,K]^T (+ epilogue). x, out 2-D row-major (unit inner stride)."""
    m, k = x.shape
    n = w.shape[0]
    return gemm(x, w, out, m, n, k, lda=x.stride(0), ldb=w.stride(0), ldc=out.stride(0), bias=bias, **kw)


def linear_dgrad(dy, w, out, **kw):
    """out[M,K] = dy[M,N] . w[N,K]"""
    m, n = dy.shape
    k = w.shape[1]
    return gemm(dy, w, out, m, k, n, lda=dy.stride(0), ldb=w.stride(0), ldc=out.stride(0), b_trans=True, **kw)


def wgrad_plan(n_out, k_in, rows):
    """Tile and split-K for dW = dY^T X (reduction over the B*T rows): 128x128 tiles, splits chosen so that
    ~320 workgroups fill the 256 CUs while each split keeps >= 256 rows."""
    if n_out == 64 and k_in % 64 == 0 and k_in <= 576 and rows >= 64 * 256:
        return 64, 256   # gemm.hip tall-K kernel (conv2 dW): one 64 x k_in partial per split, 256 splits
    tile = 128 if (n_out >= 128 and k_in >= 128) else 64
    tiles = math.ceil(n_out / tile) * math.ceil(k_in / tile)
    splitk = 1
    if tiles < 256:
        splitk = max(1, min(rows // 256, round(320 / tiles), 256))
    return tile, splitk


def linear_wgrad(dy, x, wgrad, *, beta=1.0, bias_grad=None, **kw):
    """wgrad[N,K] (+)= dy[M,N]^T . x[M,K]  (fp32 gradient buffer); bias_grad[N] (+)= colsum(dy) fused into
    the same GEMM (bf16 operands) or a separate native reduction (fp32 parity path)."""
    m, n = dy.shape
    k = x.shape[1]
    tile, splitk = wgrad_plan(n, k, m)
    if dy.dtype != torch.bfloat16:
        tile = 0
    fuse = bias_grad is not None and dy.dtype == torch.bfloat16
    ws = gemm(dy, x, wgrad, n, k, m, lda=dy.stride(0), ldb=x.stride(0), ldc=wgrad.stride(0), a_trans=True,
              b_trans=True, beta=beta, splitk=kw.pop("splitk", splitk), tile=kw.pop("tile", tile),
              rowsum=bias_grad if fuse else None, **kw)
    if bias_grad is not None and not fuse:
        colsum(dy, bias_grad)
    return ws


GROUPED_TABLE_KERNEL = "gemm_bf16_grouped_dev_kernel<true, true>"
# (beta != 1, beta == 1) instantiations (96 = E_BETA | E_F32: accumulate into the fp32 grads)
GROUPED_P3_KERNELS = ("gemm_bf16_p3g_kernel<64>", "gemm_bf16_p3g_kernel<96>")
GROUPED_P4_KERNELS = ("gemm_bf16_p4g_kernel<64>", "gemm_bf16_p4g_kernel<96>")
GROUPED_WS_KERNELS = ("gemm_bf16_wsg_kernel<64>", "gemm_bf16_wsg_kernel<96>")
GROUPED_WSQ_KERNELS = ("gemm_bf16_wsgq_kernel<64>", "gemm_bf16_wsgq_kernel<96>")
GROUPED_WSQA_KERNELS = ("gemm_bf16_wsgqa_kernel<64>", None)   # AdamW fused (beta 0 only)
GROUPED_FUSED_KERNELS = {GROUPED_WSQA_KERNELS[0]}


def wgrad_groupable(dy, x, wgrad):
    """Can dW (+)= dy^T x join a grouped launch (bf16, 16-byte aligned rows, fp32 grads, moderate K)?"""
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and wgrad.dtype == torch.float32
            and dy.stride(1) == 1 and x.stride(1) == 1 and wgrad.stride(1) == 1
            and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0
            and x.data_ptr() % 16 == 0 and dy.shape[0] <= 65536)


# Weight-gradient kernel: "ws" = the warp-specialised 256x128 tiles (gemm_ws.hip: 4 MFMA waves + 4 LDS-DMA loader
# waves, 3-stage ring, bias-gradient row sums on the loader waves; c3 step 13.55-13.61 -> 13.06-13.13 ms against
# "p4", same box, alternating), "p4" = 256x256 tiles on the software-pipelined LDS-DMA ring (gemm.hip p4_body),
# "p3" = the 256x128 ring, "reg" = the register-staged 128x128 tiles (also the fallback for tables the rings
# cannot take).  ASRX_WGRAD_KIND overrides.
WGRAD_KIND = os.environ.get("ASRX_WGRAD_KIND", "ws")


def _grouped_p3_ok(items, beta):
    """Can the LDS-DMA ring kernel take these weight gradients (fp32 C rows 16-byte aligned, beta 0 or 1)?"""
    return WGRAD_KIND in ("p3", "p4", "ws") and beta in (0.0, 1.0) and all(
        x.shape[1] % 4 == 0 and wgrad.stride(0) % 4 == 0 and wgrad.data_ptr() % 16 == 0
        for (_, x, wgrad, _) in items)


_XCD_PLANS = {}


def xcd_plan(shapes, tile=256, nxcd=8, pack=None):
    """Lay grouped weight-gradient tiles out over the 8 XCDs (workgroup b runs on XCD b % 8): whole groups
    (longest reductions, then largest groups first) go to the least-loaded XCD, so the tiles of a group run on
    one XCD at the same time and share its L2, and every XCD gets about the same work.
    pack (default WGRAD_PACK): additionally pack the groups into rounds of 32 tiles — one workgroup per CU,
    32 CUs per XCD — so that a group never straddles two rounds (the tiles of a straddling group run a whole
    reduction apart and fetch their shared operand panels twice).
    shapes: (m, n, k) per group (C[m,n], reduction k).  Returns (group order, tiles per group, block -> tile map)."""
    import numpy as np
    pack = WGRAD_PACK if pack is None else pack
    key = (tuple(shapes), tile, nxcd, pack)
    if key in _XCD_PLANS:
        return _XCD_PLANS[key]
    tm, tn = tile if isinstance(tile, tuple) else (tile, tile)
    nts = [((m + tm - 1) // tm) * ((n + tn - 1) // tn) for (m, n, k) in shapes]
    order = sorted(range(len(shapes)), key=lambda i: (-shapes[i][2], -nts[i], i))
    load = [0] * nxcd
    if not pack or nxcd == 1:
        per_xcd = [[] for _ in range(nxcd)]
        for i in order:
            x = min(range(nxcd), key=lambda j: (load[j], j))
            per_xcd[x].append(i)
            load[x] += nts[i] * shapes[i][2]
        group_order = [i for x in range(nxcd) for i in per_xcd[x]]
        first = {}
        t = 0
        for i in group_order:
            first[i] = t
            t += nts[i]
        slots = [[first[i] + j for i in per_xcd[x] for j in range(nts[i])] for x in range(nxcd)]
    else:
        cap = 32   # CUs per XCD
        group_order = order
        first = {}
        t = 0
        for i in group_order:
            first[i] = t
            t += nts[i]
        # chunks of <= cap consecutive tiles (they share operand panel rows), first-fit decreasing into
        # same-reduction bins of cap tiles
        chunks = [(shapes[i][2], i, t0, min(nts[i], t0 + cap)) for i in order for t0 in range(0, nts[i], cap)]
        chunks.sort(key=lambda c: (-c[0], -(c[3] - c[2]), c[1], c[2]))
        bins = []   # [k, fill, chunks]
        for c in chunks:
            size = c[3] - c[2]
            for b in bins:
                if b[0] == c[0] and b[1] + size <= cap:
                    b[1] += size
                    b[2].append(c)
                    break
            else:
                bins.append([c[0], size, [c]])
        # longest reductions first, full rounds before partial ones (a partial round lets the next one start early)
        bins.sort(key=lambda b: (-b[0], -b[1]))
        slots = [[] for _ in range(nxcd)]
        for b in bins:
            x = min(range(nxcd), key=lambda j: (load[j], j))
            slots[x].extend(first[i] + j for (_, i, t0, t1) in b[2] for j in range(t0, t1))
            load[x] += b[1] * b[0]
    depth = max(len(sl) for sl in slots)
    block_tile = np.full(depth * nxcd, 0xFFFF, dtype=np.uint16)
    for x in range(nxcd):
        block_tile[x:x + nxcd * len(slots[x]):nxcd] = slots[x]
    tmap = np.concatenate([np.full(nts[i], slot, dtype=np.uint16) for slot, i in enumerate(group_order)])
    plan = (group_order, nts, block_tile, tmap)
    _XCD_PLANS[key] = plan
    return plan


_TILE_CODE = {"p3": ((256, 128), 3), "p4": ((256, 256), 4), "ws": ((256, 128), 5), "reg": ((128, 128), 128)}


def upload(dst, host_bytes):
    """Host bytes -> device tensor `dst` on the current stream through kernel arguments (asrx_upload): no pinned
    staging buffer, capturable in a HIP graph."""
    import numpy as np
    buf = np.ascontiguousarray(host_bytes).view(np.uint8)
    call("asrx_upload", dst.data_ptr(), buf.ctypes.data, buf.nbytes, stream())


_CONST_MAPS = {}   # (id of a cached xcd_plan tile map, device) -> (device copy of tile map + block map, offset, tmap)


def _grouped_xcd(items, common, kind="p3", adam=None):
    """Grouped weight gradients with an XCD-aware workgroup -> tile map (asrx_gemm_grouped_xcd): 64-B group
    entries (operand pointers: per call), then the tile -> group and block -> tile maps (per shape set, cached on
    the host), written into one device buffer by asrx_upload.  Returns (flops, launch(), table buffer): the
    caller issues launch() right away (stream-ordered reuse then makes dropping the buffer safe)."""
    import numpy as np
    shapes = [(dy.shape[1], x.shape[1], dy.shape[0]) for (dy, x, _, _) in items]
    tile, code = _TILE_CODE[kind]
    group_order, nts, block_tile, tmap = xcd_plan(shapes, tile=tile, nxcd=8 if WGRAD_XCD else 1)
    common.tile = code
    cvec = 1
    ents = np.zeros((len(items), 8), dtype=np.int64)
    ints = ents.view(np.int32)
    start, flops, panels = 0, 0, 0
    for slot, i in enumerate(group_order):
        dy, x, wgrad, bias_grad = items[i]
        _cuda(dy, x, wgrad, bias_grad)
        m, n = dy.shape
        k = x.shape[1]
        ents[slot, 0], ents[slot, 1], ents[slot, 2] = dy.data_ptr(), x.data_ptr(), wgrad.data_ptr()
        ents[slot, 3] = bias_grad.data_ptr() if bias_grad is not None else 0
        # last field: the group's first row-panel counter (ws queue launch: split bias-gradient row sums)
        ints[slot, 8:16] = [dy.stride(0), x.stride(0), wgrad.stride(0), n, k, m, start, panels]
        if bias_grad is not None:
            panels += (n + tile[0] - 1) // tile[0]
        start += nts[i]
        flops += 2 * m * n * k
        if wgrad.stride(0) % 4 or wgrad.data_ptr() % 16:
            cvec = 0
    common.relu = cvec
    queue = code == 5 and WGRAD_QUEUE and len(block_tile) % 8 == 0
    dev_ = items[0][0].device
    # the tile -> group and block -> tile maps depend on the shapes only: one device copy per plan, written outside
    # any graph capture and reused by every later call (a captured graph's launches point at it), so a step uploads
    # just the group entries and the zeroed counters (round 5: 7 -> 3 upload launches per c3 step)
    cmaps = _CONST_MAPS.get((id(tmap), dev_))
    if cmaps is None and not torch.cuda.is_current_stream_capturing():
        ob = (tmap.nbytes + 63) // 64 * 64
        hostc = np.zeros((ob + block_tile.nbytes + 3) // 4 * 4, dtype=np.uint8)
        hostc[:tmap.nbytes] = tmap.view(np.uint8)
        hostc[ob:ob + block_tile.nbytes] = block_tile.view(np.uint8)
        cdev = torch.empty(hostc.size, dtype=torch.uint8, device=dev_)
        upload(cdev, hostc)
        cmaps = _CONST_MAPS[(id(tmap), dev_)] = (cdev, ob, tmap)   # (tmap kept: its id stays unique)
    o1 = (ents.nbytes + 63) // 64 * 64
    if cmaps is not None:
        # per call: group entries, then (ws queue) 8 per-XCD queue counters (+ 8 spare) and one counter per
        # bias-carrying row panel, zeroed by this upload, i.e. on every launch / replay
        n_all = o1 + 4 * (16 + panels) if queue else o1
        host = np.zeros(n_all, dtype=np.uint8)
        host[:ents.nbytes] = ents.view(np.uint8).reshape(-1)
        dev = torch.empty(n_all, dtype=torch.uint8, device=dev_)
        upload(dev, host)
        base = dev.data_ptr()
        tg, bt, ctr = cmaps[0].data_ptr(), cmaps[0].data_ptr() + cmaps[1], base + o1
    else:   # (first sight of this plan inside a capture: everything in one per-call buffer, as in round 4)
        o2 = o1 + (tmap.nbytes + 63) // 64 * 64
        o3 = (o2 + block_tile.nbytes + 63) // 64 * 64
        n_all = o3 + 4 * (16 + panels) if queue else (o2 + block_tile.nbytes + 3) // 4 * 4
        host = np.zeros(n_all, dtype=np.uint8)
        host[:ents.nbytes] = ents.view(np.uint8).reshape(-1)
        host[o1:o1 + tmap.nbytes] = tmap.view(np.uint8)
        host[o2:o2 + block_tile.nbytes] = block_tile.view(np.uint8)
        dev = torch.empty(n_all, dtype=torch.uint8, device=dev_)
        upload(dev, host)
        base = dev.data_ptr()
        tg, bt, ctr = base + o1, base + o2, base + o3
    part = None
    if queue:
        common.workspace, common.workspace_elems = ctr, 16 + panels
        part = torch.empty(start * tile[0], dtype=torch.float32, device=dev.device)
        common.rowsum_ws = part.data_ptr()

    fused = adam is not None and queue and common.beta == 0.0

    def launch():
        if fused:   # (the AdamDesc is held by this closure until the call)
            call("asrx_gemm_grouped_xcd_adam", ctypes.byref(common), base, tg, bt, len(items), start,
                 len(block_tile), ctypes.byref(adam), stream())
        else:
            call("asrx_gemm_grouped_xcd", ctypes.byref(common), base, tg, bt, len(items), start,
                 len(block_tile), stream())
    return flops, launch, (dev, part), (queue, fused)


# lay each group's tiles on one XCD (False: one table order over all XCDs; module constants the tests patch — their
# environment switches were removed in round 5)
WGRAD_XCD = True
# pack the groups into 32-tile rounds per XCD (xcd_plan; False: whole groups per XCD).  Neutral for
# the single-GPU step's one grouped launch (13.37-13.40 ms either way), but a multi-GPU backward's decoder release
# launch is the cross K/V group (96 long tiles) plus short decoder tiles: whole groups put all 96 on one XCD's 32 CUs
# (three rounds, modelled makespan 747 K-steps) where packed 32-tile chunks spread them (313)
WGRAD_PACK = True
# ws grouped launch from persistent workgroups on per-XCD tile queues (False: one workgroup per tile, started by the
# in-order dispatcher)
WGRAD_QUEUE = True


def linear_wgrad_grouped(items, *, beta=1.0, kind=None, adam=None):
    """Issue many independent weight gradients wgrad[N,K] (+)= dy[M,N]^T . x[M,K] (+ bias_grad[N] += colsum dy)
    as ONE grouped launch (longest reductions first, tiles of a group on one XCD).  adam (AdamDesc, optional): the
    AdamW step of every written element fused into the launch (asrx_gemm_grouped_xcd_adam) where the launch can take
    it (ws queue launch, beta 0).  Returns the name of the kernel instantiation launched (the one rocprofv3 lists);
    it is in GROUPED_FUSED_KERNELS exactly when the optimizer step was fused."""
    if not items:
        return None
    items = sorted(items, key=lambda it: -it[0].shape[0])
    common = GemmDesc()
    common.in_dtype, common.a_trans, common.b_trans, common.c_dtype = BF16, 1, 1, F32
    common.alpha, common.beta = 1.0, beta
    p3 = _grouped_p3_ok(items, beta)
    kind = kind or WGRAD_KIND
    # the table upload is issued first, so a timed bracket holds the grouped GEMM alone
    flops, launch, _, (queued, fused) = _grouped_xcd(items, common, kind if p3 else "reg",
                                                     adam if p3 and kind == "ws" else None)
    # the kernel that actually runs: the ws tiles go to the persistent queue kernel only when _grouped_xcd took it
    # (its block map must hold whole 8-XCD rounds), else one workgroup per tile
    wsk = GROUPED_WSQA_KERNELS if fused else GROUPED_WSQ_KERNELS if queued else GROUPED_WS_KERNELS
    kname = ({"p4": GROUPED_P4_KERNELS, "ws": wsk}.get(kind, GROUPED_P3_KERNELS)[beta == 1.0] if p3
             else GROUPED_TABLE_KERNEL)
    probe = PROBE
    if probe is not None:
        # algorithmic bytes: every operand panel once (bf16 dY and X, each distinct tensor counted once), the fp32 dW /
        # db stores (+ their reads for beta 1), and with the optimizer fused 26 B more per parameter (fp32 master and
        # both moments read and written, the bf16 shadow written)
        seen, nb = set(), 0
        for dy, x, gw, gb in items:
            for t in (dy, x):
                if t.data_ptr() not in seen:
                    seen.add(t.data_ptr())
                    nb += t.shape[0] * t.shape[1] * t.element_size()
            for t in (gw, gb):
                if t is not None:
                    nb += t.numel() * 4 * (2 if beta == 1.0 else 1) + (26 * t.numel() if fused else 0)
        probe.alg_bytes[kname] = nb
    if probe is not None and probe.active and probe.log is not None:
        probe.log.append((kname, len(items), 0,
                          sum(it[0].shape[0] * it[0].shape[1] * it[1].shape[1] for it in items), 1, 1))
    if probe is not None and probe.active:
        timed_launch(kname, flops, launch)
    else:
        launch()
    return kname


def colsum(x, out, *, accumulate=True, rows=None, cols=None, ld=None):
    """out[c] (+)= sum_r x[r, c]"""
    _cuda(x, out)
    rows = x.shape[0] if rows is None else rows
    cols = x.shape[1] if cols is None else cols
    ld = x.stride(0) if ld is None else ld
    nblocks = max(1, min(512, (rows + 63) // 64))
    part = torch.empty(nblocks * cols, device=x.device, dtype=torch.float32)
    call("asrx_reduce_rows", code(x), x.data_ptr(), rows, cols, ld, out.data_ptr(), int(accumulate),
         part.data_ptr(), nblocks, stream())


# ------------------------------------------------------------------------------------------- LayerNorm

def layernorm_fwd(x, gamma, beta, y, eps=1e-5):
    _cuda(x, gamma, beta, y)
    rows, d = x.shape
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    call("asrx_layernorm_fwd", code(x), x.data_ptr(), code(y), y.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), rows, d, eps, stream())
    return mean, rstd


def reduce_rows_grouped(items):
    """out (+)= column sums of fp32 [rows, cols] matrices, many per launch: items = [(in, out, accumulate)]."""
    for c0 in range(0, len(items), MAX_ROWSUM_GROUPS):
        chunk = items[c0:c0 + MAX_ROWSUM_GROUPS]
        arr = (RowsumGroup * len(chunk))()
        for gr, (src, out, acc) in zip(arr, chunk):
            _cuda(src, out)
            gr.in_, gr.rows, gr.cols = src.data_ptr(), src.shape[0], src.shape[1]
            gr.out, gr.accumulate = out.data_ptr(), int(acc)
        call("asrx_reduce_rows_grouped", arr, len(chunk), stream())


LN_BWD_BLOCKS = 512   # (tools/ln_bench.py: 26.1-26.6 us cold vs 26.7 at 1024; 256 measured equal in the step)
LN_BWD512_WAVES = 8   # waves per block of the d = 512 kernel (norm.hip LNB_W): half the blocks for the same waves


def layernorm_bwd(x, dy, gamma, mean, rstd, dgb, *, dres=None, dx_drop=None, dropout_p=0.0, seed=0, defer=None):
    """Returns dx (fp32). dgb: fp32 [2*d] grad buffer (gamma grads then beta grads), accumulated.
    If dx_drop (bf16 or fp32) is given it receives dropout_bwd(dx) for the upstream sublayer.  With a `defer`
    list the per-block dgamma|dbeta partials are queued for reduce_rows_grouped instead of reduced here."""
    _cuda(x, dy, gamma, mean, rstd, dgb)
    rows, d = x.shape
    dx = torch.empty(rows, d, device=x.device, dtype=torch.float32)
    wpb = LN_BWD512_WAVES if d == 512 else 4   # (the d = 512 kernel's blocks hold 8 waves)
    nblocks = max(1, min(LN_BWD_BLOCKS * 4 // wpb, (rows + 2 * wpb - 1) // (2 * wpb)))   # >= 2 rows per wave
    part = torch.empty(nblocks * 2 * d, device=x.device, dtype=torch.float32)
    call("asrx_layernorm_bwd", code(x), x.data_ptr(), code(dy), dy.data_ptr(), gamma.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), _p(dres), dx.data_ptr(), _p(dx_drop), code(dx_drop) if dx_drop is not None else 0,
         dropout_p, seed & _U64, part.data_ptr(), nblocks, rows, d, stream())
    if defer is not None:
        defer.append((part.view(nblocks, 2 * d), dgb, True))
        return dx
    part2 = torch.empty(max(1, (nblocks + 63) // 64) * 2 * d, device=x.device, dtype=torch.float32)
    call("asrx_reduce_rows", F32, part.data_ptr(), nblocks, 2 * d, 2 * d, dgb.data_ptr(), 1, part2.data_ptr(),
         max(1, (nblocks + 63) // 64), stream())
    return dx


# ------------------------------------------------------------------------------------------- attention

class MaskSpec:
    """How a score (b, q, key) is masked (True = -inf). mode 0: none; 1: causal/key-valid/query-valid vectors;
    2: dense bytes with broadcast strides."""

    def __init__(self, mode=0, causal=False, kvalid=None, qvalid=None, valid_bstride=0, dense=None,
                 strides=(0, 0, 0)):
        self.mode, self.causal = mode, causal
        self.kvalid, self.qvalid, self.valid_bstride = kvalid, qvalid, valid_bstride
        self.dense, self.strides = dense, strides

    @staticmethod
    def decoder(mask):
        """model.py:108-115: pad = mask < 1; masked = causal | key pad | query pad."""
        valid = (mask >= 1).to(torch.uint8).contiguous()
        return MaskSpec(1, True, valid, valid, valid.stride(0))

    @staticmethod
    def from_attention_mask(m, B, Lq, Lk):
        """Any-dtype mask broadcastable to (B, Lq, Lk); nonzero (>0) means masked (layers.py:22-23)."""
        if m is None:
            return MaskSpec()
        mb = m.gt(0).to(torch.uint8)
        while mb.dim() < 3:
            mb = mb.unsqueeze(0)
        mb = mb.expand(B, Lq, Lk)
        return MaskSpec(2, dense=mb, strides=tuple(mb.stride()))


def _attn_desc(q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, dropout_p, seed):
    d = AttnDesc()
    d.batch, d.heads, d.lq, d.lk, d.dh = B, H, Lq, Lk, dh
    (qr, qb), (kr, kb), (vr, vb), (orr, ob) = strides
    d.q, d.q_rstride, d.q_bstride = q.data_ptr(), qr, qb
    d.k, d.k_rstride, d.k_bstride = k.data_ptr(), kr, kb
    d.v, d.v_rstride, d.v_bstride = v.data_ptr(), vr, vb
    d.o, d.o_rstride, d.o_bstride = o.data_ptr(), orr, ob
    d.scale = scale
    d.mask_mode, d.causal = spec.mode, int(spec.causal)
    d.kvalid, d.qvalid, d.valid_bstride = _p(spec.kvalid), _p(spec.qvalid), spec.valid_bstride
    if spec.mode == 2:
        d.mask = spec.dense.data_ptr()
        d.mask_sb, d.mask_sq, d.mask_sk = spec.strides
    d.dropout_p, d.seed = dropout_p, seed & _U64
    return d


def qmaj_stride(Lk):
    """Row stride (32-bit words) of the query-major keep bits: ceil(Lk / 32) up to 256 keys, rounded up to a
    multiple of 4 past that (the streamed forward moves 4 words per query and 128-key chunk)."""
    nkw = (Lk + 31) // 32
    return nkw if Lk <= 256 else (nkw + 3) // 4 * 4


def dropmask_buffer(B, H, Lq, Lk, dh, dropout_p, device):
    """Keep-bit buffer the fused attention forward fills for its backward (None when unused): key-major words
    [B*H][ceil(Lq/32)][Lk], then query-major words [B*H][Lq][qmaj_stride(Lk)]."""
    if dropout_p <= 0.0 or dh != 64:
        return None
    from ._lib import lib
    n = lib().asrx_attn_dropmask_words(B, H, Lq, Lk)   # the C-ABI's own size rule (include/asrx.h)
    assert n == B * H * (((Lq + 31) // 32) * Lk + Lq * qmaj_stride(Lk)), (n, B, H, Lq, Lk)
    return torch.empty(n, device=device, dtype=torch.int32)


def attention_dropgen(B, H, Lq, Lk, dh, dropout_p, seed, dropmask):
    """Generate the attention dropout keep bits into `dropmask` (see dropmask_buffer) on the current stream."""
    _cuda(dropmask)
    d = AttnDesc()
    d.batch, d.heads, d.lq, d.lk, d.dh = B, H, Lq, Lk, dh
    d.q = d.k = d.v = dropmask.data_ptr()      # not read; fill_args only checks them
    d.dropout_p, d.seed = dropout_p, seed & _U64
    d.dropmask = dropmask.data_ptr()
    call("asrx_attn_dropgen", ctypes.byref(d), stream())


def layernorm_fwd_dropgen(x, gamma, beta, y, B, H, Lq, Lk, dh, dropout_p, seed, dropmask, eps=1e-5):
    """layernorm_fwd (x fp32 [rows, 512] -> y bf16) and attention_dropgen in ONE launch (asrx_layernorm_fwd_attn_dropgen):
    the keep-bit hashing runs beside the HBM-bound LayerNorm.  Returns (mean, rstd)."""
    _cuda(x, gamma, beta, y, dropmask)
    rows, d = x.shape
    # the fused kernel indexes rows as row * 512 with 16-B vectors: dense [rows, 512] fp32 in, bf16 out only
    if not (d == 512 and x.dtype == torch.float32 and y.dtype == torch.bfloat16 and x.is_contiguous()
            and y.is_contiguous() and y.shape == x.shape and gamma.is_contiguous() and beta.is_contiguous()
            and gamma.numel() == d and beta.numel() == d and gamma.data_ptr() % 16 == 0 and beta.data_ptr() % 16 == 0):
        raise RuntimeError("asrx.layernorm_fwd_dropgen: needs contiguous [rows, 512] fp32 x / bf16 y and 16-B aligned "
                           "gamma/beta")
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    a = AttnDesc()
    a.batch, a.heads, a.lq, a.lk, a.dh = B, H, Lq, Lk, dh
    a.q = a.k = a.v = dropmask.data_ptr()      # not read; fill_args only checks them
    a.dropout_p, a.seed = dropout_p, seed & _U64
    a.dropmask = dropmask.data_ptr()
    call("asrx_layernorm_fwd_attn_dropgen", x.data_ptr(), y.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), rows, d, eps, ctypes.byref(a), stream())
    return mean, rstd


def attention_fwd(q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, dropout_p=0.0, seed=0, dropmask=None,
                  dropmask_ready=False, o_lo=None):
    """Fused attention (bf16). Returns lse [B*H*Lq] (log2 domain).  o_lo (optional, bf16, o's strides): receives
    the rounding residual O - bf16(O) for an exact backward delta (training)."""
    _cuda(q, k, v, o, dropmask, o_lo)
    lse = torch.empty(B * H * Lq, device=q.device, dtype=torch.float32)
    d = _attn_desc(q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, dropout_p, seed)
    d.lse = lse.data_ptr()
    d.dropmask = _p(dropmask)
    d.dropmask_ready = int(bool(dropmask_ready))
    d.o_lo = _p(o_lo)
    call("asrx_attention_fwd", ctypes.byref(d), stream())
    return lse


def attention_bwd(q, k, v, o, lse, do, dq, dk, dv, B, H, Lq, Lk, dh, strides, gstrides, scale, spec,
                  dropout_p=0.0, seed=0, dropmask=None, o_lo=None):
    _cuda(q, k, v, o, lse, do, dq, dk, dv, dropmask, o_lo)
    d = _attn_desc(q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, dropout_p, seed)
    d.lse = lse.data_ptr()
    d.dropmask = _p(dropmask)
    d.o_lo = _p(o_lo)
    (dor, dob), (dqr, dqb), (dkr, dkb), (dvr, dvb) = gstrides
    d.dout, d.do_rstride, d.do_bstride = do.data_ptr(), dor, dob
    d.dq, d.dq_rstride, d.dq_bstride = dq.data_ptr(), dqr, dqb
    d.dk, d.dk_rstride, d.dk_bstride = dk.data_ptr(), dkr, dkb
    d.dv, d.dv_rstride, d.dv_bstride = dv.data_ptr(), dvr, dvb
    delta = torch.empty(B * H * Lq, device=q.device, dtype=torch.float32)
    d.delta = delta.data_ptr()
    acc = None
    from ._lib import lib
    nacc = lib().asrx_attn_dq_acc_elems(B, H, Lq, Lk, dh)   # fp32 dQ partials, one per key block (asrx.h dq_acc)
    if nacc < 0:
        raise RuntimeError(f"asrx.attention_bwd: bad shapes {(B, H, Lq, Lk, dh)}")
    if nacc > 0:
        acc = torch.empty(nacc, device=q.device, dtype=torch.float32)
        d.dq_acc = acc.data_ptr()
    call("asrx_attention_bwd", ctypes.byref(d), stream())


def softmax_fwd(s, p, pd, nbh, H, Lq, Lk, ld, scale, spec, dropout_p=0.0, seed=0):
    _cuda(s, p, pd)
    sb, sq, sk = spec.strides if spec.mode == 2 else (0, 0, 0)
    call("asrx_softmax_fwd", code(s), s.data_ptr(), p.data_ptr(), _p(pd), nbh, H, Lq, Lk, ld, scale, spec.mode,
         int(spec.causal), _p(spec.kvalid), _p(spec.qvalid), spec.valid_bstride,
         _p(spec.dense) if spec.mode == 2 else None, sb, sq, sk, dropout_p, seed & _U64, stream())


def softmax_bwd(p, dpd, ds, nbh, Lq, Lk, ld, scale, dropout_p=0.0, seed=0):
    _cuda(p, dpd, ds)
    call("asrx_softmax_bwd", code(p), p.data_ptr(), dpd.data_ptr(), ds.data_ptr(), nbh, Lq, Lk, ld, scale,
         dropout_p, seed & _U64, stream())


# ------------------------------------------------------------------------------------------- misc

def cast(src, dst):
    _cuda(src, dst)
    assert src.numel() == dst.numel()
    call("asrx_cast", code(src), src.data_ptr(), code(dst), dst.data_ptr(), src.numel(), stream())


EW_RELU_GRAD, EW_DROPOUT, EW_ADD = 0, 1, 2


def ewise(op, a, out, b=None, p=0.0, seed=0):
    """out = op(a, b) elementwise over contiguous tensors of equal size (asrx_ewise; fp32 / bf16, may alias):
    EW_RELU_GRAD (b > 0 ? a : 0), EW_DROPOUT (keep(seed, i) ? a / (1 - p) : 0), EW_ADD (a + b)."""
    _cuda(a, b, out)
    n = a.numel()
    assert out.numel() == n and (b is None or b.numel() == n)
    assert a.is_contiguous() and out.is_contiguous() and (b is None or b.is_contiguous())
    call("asrx_ewise", op, code(a), a.data_ptr(), code(b) if b is not None else 0, _p(b), code(out), out.data_ptr(),
         n, float(p), seed & _U64, stream())


def greedy_argmax(logits, V, tok_col, cur=None):
    """tok_col[r] (a strided int64 column view) = cur[r] = first argmax of logits[r, :V] (fp32 [rows, ld])."""
    _cuda(logits, tok_col, cur)
    rows = logits.shape[0]
    call("asrx_greedy_argmax", logits.data_ptr(), rows, V, logits.stride(0), tok_col.data_ptr(),
         tok_col.stride(0), _p(cur), stream())


def sum_chunks_bf16(recv, world, chunk, out):
    """out[i] = bf16(sum_w recv[w * chunk + i]) with an fp32 sum (bf16-wire gradient exchange, asrx.dist)."""
    _cuda(recv, out)
    call("asrx_sum_chunks_bf16", recv.data_ptr(), world, chunk, out.data_ptr(), stream())


def zero_spans(buf, spans):
    """buf[a:b] = 0 for every row (a, b) of the device int64 table `spans` [n, 2] (asrx_zero_spans)."""
    _cuda(buf, spans)
    assert buf.dtype == torch.float32 and spans.dtype == torch.int64 and spans.is_contiguous()
    call("asrx_zero_spans", buf.data_ptr(), spans.data_ptr(), spans.shape[0], stream())


ROW_SCALE, ROW_ADD = 0, 1


def rowwise(op, a, b, out, period=1):
    """fp32 [rows, d]: ROW_SCALE out = a * b[:, None] (b [rows]); ROW_ADD out = a + b[r % period] (b [period, d])
    (asrx_rowwise; out may alias a)."""
    _cuda(a, b, out)
    assert a.dtype == b.dtype == out.dtype == torch.float32 and a.is_contiguous() and out.is_contiguous()
    assert b.is_contiguous() and out.shape == a.shape and a.dim() == 2
    rows, d = a.shape
    assert (b.numel() == rows) if op == ROW_SCALE else (b.shape[-1] == d and b.numel() >= period * d)
    call("asrx_rowwise", op, a.data_ptr(), b.data_ptr(), out.data_ptr(), rows, d, period, stream())


def transpose_last2(x, out):
    """out[b] = x[b]^T for fp32 x (B, R, C) contiguous -> out (B, C, R) (asrx_transpose_last2)."""
    _cuda(x, out)
    assert x.dtype == out.dtype == torch.float32 and x.is_contiguous() and out.is_contiguous() and x.dim() == 3
    B, R, C = x.shape
    assert out.shape == (B, C, R)
    call("asrx_transpose_last2", x.data_ptr(), B, R, C, out.data_ptr(), stream())


def step_tokens(text, inp, mask):
    """(dec_in int64 [B*L], tgt int64 [B*L], valid uint8 [B, L]) of a teacher-forced step from (B, L+1) token rows
    and the float pad mask (asrx_step_tokens): inp[:, :-1], text[:, 1:], mask[:, :-1] >= 1."""
    _cuda(text, inp, mask)
    assert text.dtype == torch.int64 and inp.dtype == torch.int64 and mask.dtype == torch.float32
    assert text.stride(1) == 1 and inp.stride(1) == 1 and mask.stride(1) == 1 and text.shape == inp.shape == mask.shape
    B, L = text.shape[0], text.shape[1] - 1
    dec_in = torch.empty(B * L, dtype=torch.int64, device=text.device)
    tgt = torch.empty(B * L, dtype=torch.int64, device=text.device)
    valid = torch.empty(B, L, dtype=torch.uint8, device=text.device)
    call("asrx_step_tokens", text.data_ptr(), text.stride(0), inp.data_ptr(), inp.stride(0), mask.data_ptr(),
         mask.stride(0), B, L, dec_in.data_ptr(), tgt.data_ptr(), valid.data_ptr(), stream())
    return dec_in, tgt, valid


def dropout_mask(n, p, seed, device):
    keep = torch.empty(n, dtype=torch.uint8, device=device)
    call("asrx_dropout_mask", keep.data_ptr(), n, p, seed & _U64, stream())
    return keep


def conv1_fwd(x, w, b, y1, mask=None):
    """y1 = relu(conv1(x)) channels-last; mask (optional, uint8 (B, F1, T1, 8)): y1 > 0 sign bits."""
    _cuda(x, w, b, y1, mask)
    B, _, F, T = x.shape
    call("asrx_conv1_fwd", x.data_ptr(), B, F, T, w.data_ptr(), b.data_ptr(), y1.data_ptr(), code(y1), _p(mask),
         stream())


def im2col_conv2(y1, cols):
    _cuda(y1, cols)
    B, F1, T1, _ = y1.shape
    assert y1.dtype == cols.dtype
    call("asrx_im2col_conv2", code(y1), y1.data_ptr(), B, F1, T1, cols.data_ptr(), stream())


def col2im_conv2(dcols, y1, dy1):
    _cuda(dcols, y1, dy1)
    B, F1, T1, _ = y1.shape
    call("asrx_col2im_conv2", code(dcols), dcols.data_ptr(), code(y1), y1.data_ptr(), B, F1, T1, dy1.data_ptr(),
         stream())


def conv2_fwd(y1, w2, bias, out):
    """out[B*T2*F2, 64] (bf16) = relu(conv2(y1) + bias), an implicit GEMM over y1 (B, F1, T1, 64) channels-last
    bf16; w2: [64][576] bf16 with columns (kh, kw, c)."""
    _cuda(y1, w2, bias, out)
    B, F1, T1, _ = y1.shape
    call("asrx_conv2_fwd", y1.data_ptr(), w2.data_ptr(), bias.data_ptr(), out.data_ptr(), B, F1, T1, stream())


def conv2_wgrad(dy2, y1, dw, db, splitk=256):
    """dw[64][576] += dy2^T im2col(y1), db[64] += colsum(dy2) (fp32 grads) with the im2col rows gathered from y1
    (B, F1, T1, 64) bf16 on the fly (tall-K kernel, `splitk` row splits)."""
    _cuda(dy2, y1, dw, db)
    B, F1, T1, _ = y1.shape
    ws = torch.empty(splitk * 64 * 576, device=dy2.device, dtype=torch.float32)
    rws = torch.empty(splitk * 64, device=dy2.device, dtype=torch.float32) if db is not None else None
    call("asrx_conv2_wgrad", dy2.data_ptr(), y1.data_ptr(), B, F1, T1, dw.data_ptr(), _p(db), ws.data_ptr(),
         ws.numel(), _p(rws), splitk, stream())


CONV_BWD_MAXT1 = 1024   # frontend.hip CB_MAXT1 (LDS: weights of 6 taps + the row's y1 sign bits + 3 x lines)


def conv_bwd_implicit(dy2, w2, y1_mask, x, dw, db):
    """conv1 weight/bias gradients (+=) straight from the conv2 output gradient dy2 [B*T2*F2][64] (bf16, already
    ReLU-gated): the conv2 data gradient and col2im are formed on the fly (no dcols / dy1 in memory).
    w2: [64][576] bf16 (columns kh, kw, c); y1_mask (B, F1, T1, 8) uint8 from conv1_fwd; x the fp32 spectrum."""
    _cuda(dy2, w2, y1_mask, x, dw, db)
    B, _, F, T = x.shape
    nblocks = max(2, min(512, B * y1_mask.shape[1]))   # two persistent workgroups per CU
    part = torch.empty((nblocks + 128) * 640, device=x.device, dtype=torch.float32)
    call("asrx_conv_bwd_implicit", dy2.data_ptr(), w2.data_ptr(), y1_mask.data_ptr(), x.data_ptr(), B, F, T,
         part.data_ptr(), nblocks, dw.data_ptr(), db.data_ptr(), stream())


def conv1_bwd_w(x, dy1, dw, db):
    _cuda(x, dy1, dw, db)
    B, _, F, T = x.shape
    nblocks = 512
    part = torch.empty((nblocks + 128) * 640, device=x.device, dtype=torch.float32)   # + finish pass 1 rows
    call("asrx_conv1_bwd_w", x.data_ptr(), dy1.data_ptr(), B, F, T, part.data_ptr(), nblocks, dw.data_ptr(),
         db.data_ptr(), stream())


def conv1_bwd_fused(dcols, y1, x, dw, db):
    """conv1 weight/bias gradients directly from the conv2 column gradient (no dy1 tensor)."""
    _cuda(dcols, y1, x, dw, db)
    B, _, F, T = x.shape
    nblocks = (B * y1.shape[1] * 8 + 3) // 4  # 8 waves per conv1 output row (b, f1): frontend.hip CB_SEG
    part = torch.empty((nblocks + 128) * 640, device=x.device, dtype=torch.float32)   # + finish pass 1 rows
    call("asrx_conv1_bwd_fused", code(dcols), dcols.data_ptr(), code(y1), y1.data_ptr(), x.data_ptr(), B, F, T,
         part.data_ptr(), nblocks, dw.data_ptr(), db.data_ptr(), stream())


def embed_fwd(tok, table, pe, out, L, dropout_p=0.0, seed=0):
    _cuda(tok, table, pe, out)
    call("asrx_embed_fwd", tok.data_ptr(), tok.numel(), L, table.data_ptr(), table.shape[1], pe.data_ptr(),
         dropout_p, seed & _U64, out.data_ptr(), stream())


def embed_bwd(tok, dout, dtable, L, pad_id, dropout_p=0.0, seed=0):
    _cuda(tok, dout, dtable)
    call("asrx_embed_bwd", tok.data_ptr(), tok.numel(), L, dout.data_ptr(), dtable.shape[1], dtable.shape[0],
         pad_id, dropout_p, seed & _U64, dtable.data_ptr(), stream())


def cross_entropy(logits, V, target, ignore_index=-100, grad_scale=1.0, want_grad=True, want_argmax=False):
    """logits fp32 [rows, ld]; returns (loss[1], dlogits bf16 [rows, ld] or None, argmax or None)."""
    _cuda(logits, target)
    rows, ld = logits.shape
    loss = torch.empty(1, device=logits.device, dtype=torch.float32)
    dl = torch.empty(rows, ld, device=logits.device, dtype=torch.bfloat16) if want_grad else None
    am = torch.empty(rows, device=logits.device, dtype=torch.int64) if want_argmax else None
    ws = torch.empty(rows + 2, device=logits.device, dtype=torch.float32)
    call("asrx_cross_entropy", logits.data_ptr(), rows, V, logits.stride(0), target.data_ptr(), ignore_index,
         grad_scale, loss.data_ptr(), _p(dl), _p(am), ws.data_ptr(), stream())
    return loss, dl, am


def adam(p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, decoupled=False, hyp=None):
    """Fused Adam/AdamW step `step` (1-based).  hyp (optional fp32 device [3]): lr and bias corrections read by
    the kernel at run time (a replayed HIP graph; see adam_hyper)."""
    _cuda(p, g, m, v, p_bf16, hyp)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    call("asrx_adam", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _p(p_bf16), p.numel(), lr, beta1,
         beta2, eps, weight_decay, bc1, bc2, grad_scale, int(decoupled), _p(hyp), stream())


def adam_desc(p, m, v, p_bf16, g, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, decoupled=False,
              hyp=None):
    """The AdamW state of flat buffers p / m / v (+ bf16 shadow) laid out like the gradient buffer g, for a fused
    grouped weight-gradient launch (linear_wgrad_grouped(adam=...))."""
    from ._lib import AdamDesc
    _cuda(p, m, v, p_bf16, g, hyp)
    d = AdamDesc()
    d.p, d.m, d.v, d.p_bf16, d.g_base, d.hyp = p.data_ptr(), m.data_ptr(), v.data_ptr(), _p(p_bf16), g.data_ptr(), _p(hyp)
    d.lr, d.beta1, d.beta2, d.eps, d.weight_decay = lr, beta1, beta2, eps, weight_decay
    d.bias_corr1, d.bias_corr2 = 1.0 - beta1 ** step, 1.0 - beta2 ** step
    d.grad_scale, d.decoupled = grad_scale, int(decoupled)
    return d


def adam_spans(p, g, m, v, p_bf16, spans, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, decoupled=False,
               hyp=None):
    """AdamW over the element ranges of a device int64 [n, 2] table (bounds multiples of 4; asrx_adam_spans)."""
    _cuda(p, g, m, v, p_bf16, spans, hyp)
    call("asrx_adam_spans", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _p(p_bf16), spans.data_ptr(),
         spans.shape[0], lr, beta1, beta2, eps, weight_decay, 1.0 - beta1 ** step, 1.0 - beta2 ** step, grad_scale,
         int(decoupled), _p(hyp), stream())


def adam_hyper(hyp, lr, beta1, beta2, step):
    """Write step `step`'s {lr, 1 - beta1^step, 1 - beta2^step} into the device tensor hyp (asrx_upload)."""
    import numpy as np
    upload(hyp, np.array([lr, 1.0 - beta1 ** step, 1.0 - beta2 ** step], dtype=np.float32))


TUNE_KEYS = {"softmax_u": 1, "ln_rw": 2, "ln_pf": 3, "ln_bpc": 4}


def set_tuning(name, value):
    """Process-wide kernel-variant override (asrx_set_tuning): "softmax_u" in (1, 2, 4), "ln_rw" in (1, 2, 4),
    "ln_pf" in (1, 2, 4; 8 = the general LayerNorm kernels), "ln_bpc" in 1..16; 0 restores the environment /
    default choice.  Every variant computes the same values."""
    call("asrx_set_tuning", TUNE_KEYS[name], int(value))


def set_seed_offset(offset):
    """Per-step device-resident dropout seed offset (asrx_set_seed_offset), on the current stream."""
    call("asrx_set_seed_offset", int(offset) & _U64, stream())
