"""Flat parameter / gradient / bf16-shadow storage for a model.

All trainable parameters of a module are re-pointed into ONE contiguous fp32 master buffer
(``p.data`` becomes a view), their ``.grad`` into ONE fp32 gradient buffer, and (on GPU) a bf16
compute shadow is kept in a third buffer (``p._smi_bf16``).  Consequences on MI355X:
  * the optimizer is a single fused HIP launch over the whole model (csrc/kernels/optim.hip),
    which also refreshes the bf16 shadow — no multi-tensor-apply bookkeeping;
  * data-parallel gradient sync works on large contiguous buckets of the gradient buffer
    (few, big RCCL all-reduces — what xGMI rings want);
  * parameters are laid out in REVERSE registration order, so the backward pass finishes the
    front of the buffer first and bucket 0 can be all-reduced while backward continues.
Each parameter starts on a 64-element boundary (256-B aligned fp32, 128-B aligned bf16).

Reference-precision (fp32) models keep a fourth buffer on GPU, created on first use: the weights
split into three bf16 planes (``planes`` [3, numel], hi / mid / lo with p = hi + mid + lo
exactly; sparkmi/ops/planes.py), the operand format of the fp32 GEMM.  The optimizer kernel
rewrites the planes of every parameter it updates, and ``refresh_shadow`` (checkpoint loads,
data-parallel broadcasts / ZeRO gathers) re-splits them.

A module may list parameter groups to be stored back to back (``_smi_flat_groups()``): e.g. the
six decoder kv projections, which all read the encoder output, then form ONE [6*2D, D] weight
view and run as one GEMM (``concat``).  A group sits where its first-registered member would
(its gradients complete together, at the end of the decoder backward).
"""
import torch

from .. import _native

ALIGN = 64


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


class FlatParams:
    def __init__(self, module: torch.nn.Module, device=None, reverse=True, shadow=None):
        params = []
        seen = set()
        for name, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append((name, p))
        if reverse:
            params = params[::-1]
        params = self._place_groups(module, params)
        device = torch.device(device) if device is not None else (params[0][1].device if params else torch.device("cpu"))
        self.device = device
        self.names = [n for n, _ in params]
        self.params = [p for _, p in params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _round(p.numel())
        self.numel = off
        self.master = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        use_shadow = device.type == "cuda" if shadow is None else shadow
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=device) if use_shadow else None
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                self.master[o:o + n].copy_(p.data.reshape(-1).to(device=device, dtype=torch.float32))
                p.data = self.master[o:o + n].view(p.shape)
                p.grad = self.grad[o:o + n].view(p.shape)
                if self.shadow is not None:
                    p._smi_bf16 = self.shadow[o:o + n].view(p.shape)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.planes = None  # [3, numel] bf16 split planes, created by the first weight_planes()
        for p, o in zip(self.params, self.offsets):
            if device.type == "cuda" and p.dim() == 2:
                p._smi_planes_fn = self._planes_fn(p, o)
        object.__setattr__(module, "_smi_flat", self)  # checkpoint loads refresh the bf16 shadow
        # module.load_state_dict writes the master through p.data: re-derive the bf16 shadow and
        # the weight planes the fp32 GEMMs read.  Other in-place weight edits
        # (nn.init, p.data.copy_) must call refresh_shadow() themselves.
        import weakref
        ref = weakref.ref(self)

        def _refresh_after_load(mod, incompatible):
            f = ref()
            if f is not None and getattr(mod, "_smi_flat", None) is f:
                f.refresh_shadow()

        self._load_hook = module.register_load_state_dict_post_hook(_refresh_after_load)
        self.refresh_shadow()

    def _planes_fn(self, p, o):
        rows, cols = p.shape
        return lambda: self.ensure_planes()[:, o:o + rows * cols].view(3, rows, cols)

    def ensure_planes(self):
        """The [3, numel] split-plane buffer (allocated and split from the master on first use)."""
        if self.planes is None:
            self.planes = torch.empty(3, self.numel, dtype=torch.bfloat16, device=self.device)
            self.refresh_planes()
        return self.planes

    def plane_stride(self):
        return self.planes.stride(0) if self.planes is not None else 0

    def refresh_planes(self):
        """Re-split the planes from the fp32 master (after anything but the optimizer wrote it)."""
        if self.planes is None:
            return
        if _native.use_native(self.master):
            _native.C().split3(self.master.data_ptr(), 1, self.numel, self.numel, self.planes.data_ptr(), self.numel,
                               self.planes.stride(0), _native.stream())
        else:
            hi = self.master.to(torch.bfloat16)
            r = self.master - hi.float()
            mid = r.to(torch.bfloat16)
            self.planes[0].copy_(hi)
            self.planes[1].copy_(mid)
            self.planes[2].copy_((r - mid.float()).to(torch.bfloat16))

    def concat_planes(self, params):
        """[3, sum rows, cols] plane view of 2-D ``params`` stored back to back (see ``concat``)."""
        if self.concat(params) is None:
            return None
        o0, _ = self.param_range(params[0])
        rows = sum(p.shape[0] for p in params)
        cols = params[0].shape[1]
        return self.ensure_planes()[:, o0:o0 + rows * cols].view(3, rows, cols)

    @staticmethod
    def _place_groups(module, params):
        fn = getattr(module, "_smi_flat_groups", None)
        if fn is None:
            return params
        for group in fn():
            ids = [id(p) for p in group]
            pos = {id(p): i for i, (_, p) in enumerate(params)}
            if len(group) < 2 or any(i not in pos for i in ids) or len(set(ids)) != len(ids):
                continue
            if any(p.numel() % ALIGN for p in group[:-1]):  # padding would break the concat view
                continue
            members = {i: params[pos[i]] for i in ids}
            anchor = max(pos[i] for i in ids)
            before = [e for e in params[:anchor + 1] if id(e[1]) not in members]
            after = [e for e in params[anchor + 1:] if id(e[1]) not in members]
            params = before + [members[i] for i in ids] + after
        return params

    def concat(self, params):
        """(master, grad, shadow) views spanning ``params`` stored back to back in this order, as
        flat 1-D tensors; None when they are not contiguous here."""
        if not params or any(id(p) not in self.index for p in params):
            return None
        o0, _ = self.param_range(params[0])
        o = o0
        for p in params:
            if self.param_range(p)[0] != o:
                return None
            o += p.numel()
        return (self.master[o0:o], self.grad[o0:o], self.shadow[o0:o] if self.shadow is not None else None)

    def refresh_shadow(self):
        self.refresh_planes()
        if self.shadow is None:
            return
        if _native.use_native(self.master):
            _native.C().cast_f32_bf16(self.master.data_ptr(), self.shadow.data_ptr(), self.numel, _native.stream())
        else:
            self.shadow.copy_(self.master.to(torch.bfloat16))

    def zero_grad(self):
        self.grad.zero_()

    def param_range(self, p):
        i = self.index[id(p)]
        return self.offsets[i], self.offsets[i] + p.numel()

    def nbytes(self):
        return self.master.numel() * 4

    def state_dict_view(self):
        return {n: p for n, p in zip(self.names, self.params)}
