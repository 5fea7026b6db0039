"""Flat parameter / gradient / bf16-shadow storage.

All parameters of a model live in ONE contiguous fp32 buffer (each region 256-byte aligned); gradients in a
second one (views bound to `p.grad`), and the bf16 operand copies the MFMA GEMMs read in a third.  One cast
kernel refreshes the shadow, one fused Adam kernel updates everything, and the DDP all-reduce runs over
contiguous buckets of the gradient buffer (no per-parameter copies).

Layout hooks: a parameter may carry `_asrx_phys = (shape, perm)`: its memory is laid out as `shape` and the
logical tensor is `view(shape).permute(perm)` (e.g. the conv2 weight is stored (cout, kh, kw, cin) so that
it is the [64][576] GEMM operand of the im2col rows without a copy).
"""
import torch

ALIGN = 64  # elements


class FlatParams:
    def __init__(self, params, device):
        self.params = list(params)
        self.device = torch.device(device)
        offs, total = [], 0
        for p in self.params:
            total = (total + ALIGN - 1) // ALIGN * ALIGN
            offs.append(total)
            total += p.numel()
        total = (total + ALIGN - 1) // ALIGN * ALIGN
        self.total = total
        self.offsets = {id(p): o for p, o in zip(self.params, offs)}
        self.flat = torch.zeros(total, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(total, device=self.device, dtype=torch.float32)
        self.shadow = torch.zeros(total, device=self.device, dtype=torch.bfloat16)
        with torch.no_grad():
            for p in self.params:
                v = self._view(self.flat, p)
                v.copy_(p.data.to(self.device))
                p.data = v
                p.grad = self._view(self.grad, p)
        self._shadow_version = None
        self._w16c, self._gc, self._gview = {}, {}, {}   # cached views into the flat buffers (id(p) -> view)
        self.on_grad_ready = None   # optional callback(param_list) used by the DDP bucketer

    def _view(self, buf, p):
        o = self.offsets[id(p)]
        phys = getattr(p, "_asrx_phys", None)
        if phys is None:
            return buf[o:o + p.numel()].view(p.shape)
        shape, perm = phys
        return buf[o:o + p.numel()].view(shape).permute(perm)

    def owns(self, p):
        return id(p) in self.offsets

    def valid(self):
        for p in self.params:
            o = self.offsets[id(p)]
            if p.data.data_ptr() != self.flat.data_ptr() + 4 * o:
                return False
        return True

    def offset(self, p):
        return self.offsets[id(p)]

    # ---- raw (physical) views used by kernels
    def raw(self, p, buf=None):
        buf = self.flat if buf is None else buf
        o = self.offsets[id(p)]
        return buf[o:o + p.numel()]

    def _phys2d(self, p, buf):
        phys = getattr(p, "_asrx_phys", None)
        shape = phys[0] if phys is not None else p.shape
        r = self.raw(p, buf)
        return r.view(shape[0], -1) if len(shape) > 1 else r

    def w16(self, p):
        """bf16 operand copy of p in its PHYSICAL layout (as a 2-D [rows, cols] matrix); views cached (the flat
        buffers never move)."""
        c = self._w16c.get(id(p))
        if c is None:
            c = self._w16c[id(p)] = self._phys2d(p, self.shadow)
        return c

    def w32(self, p):
        phys = getattr(p, "_asrx_phys", None)
        shape = phys[0] if phys is not None else p.shape
        r = self.raw(p, self.flat)
        return r.view(shape[0], -1) if len(shape) > 1 else r

    def g(self, p):
        """fp32 gradient region of p (physical layout, 2-D for matrices); (re)binds p.grad if needed."""
        self.ensure_grad(p)
        c = self._gc.get(id(p))
        if c is None:
            c = self._gc[id(p)] = self._phys2d(p, self.grad)
        return c

    def span(self, first, count_params, buf):
        """A contiguous view covering `count_params` consecutive parameters starting at `first`."""
        idx = next(i for i, p in enumerate(self.params) if p is first)
        ps = self.params[idx:idx + count_params]
        o0 = self.offsets[id(ps[0])]
        o1 = self.offsets[id(ps[-1])] + ps[-1].numel()
        exp = o0
        for p in ps:
            if self.offsets[id(p)] != exp:
                return None
            exp += p.numel()
        return buf[o0:o1]

    def ensure_grad(self, p):
        v = self._gview.get(id(p))
        if v is not None and p.grad is v:
            return
        v = self._gview[id(p)] = self._view(self.grad, p)
        if p.grad is None or p.grad.data_ptr() != v.data_ptr():
            v.zero_()
        p.grad = v

    def refresh_shadow(self, force=False):
        """Re-cast the fp32 master params into the bf16 operand buffer when any param changed."""
        from .kernels import cast
        ver = sum(p._version for p in self.params)
        if force or ver != self._shadow_version:
            cast(self.flat, self.shadow)
            self._shadow_version = ver

    def mark_shadow_fresh(self):
        self._shadow_version = sum(p._version for p in self.params)

    def zero_grad(self):
        self.grad.zero_()
        for p in self.params:
            if p.grad is None:
                p.grad = self._view(self.grad, p)

    def grad_ready(self, params):
        if self.on_grad_ready is not None:
            self.on_grad_ready(params)
