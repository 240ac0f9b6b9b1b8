"""Adam step on the HIP library.

Replaces apex.FusedAdam(lr, eps=1e-15) of train_ml.py:138-153 (apex is not
available on ROCm as-is): torch.optim.Adam semantics without weight decay, one
pass per parameter tensor (rn_adam).  For the hash table the same pass writes
the f16 copy the field kernels gather from, so the next step does not need a
separate conversion.
"""
import torch

from ._lib import lib


class FusedAdam(torch.optim.Optimizer):
    # defaults as apex.FusedAdam / torch.optim.Adam: train_ml.py:143 passes
    # only lr and eps, so the reference runs betas (0.9, 0.999)
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-15, weight_decay=0.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight decay: train_ml.py uses none")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0):
        loss = closure() if closure is not None else None
        self.begin_step()
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    self.update_range(p, 0, p.numel(), grad_scale)
        self.end_step()
        return loss

    # The step in pieces, for an all-reduce epilogue (dist.GradAllReduce.
    # reduce_and_step): the step counters advance once, then each gradient
    # bucket's elements are updated as soon as its collective has landed.
    @torch.no_grad()
    def begin_step(self):
        self._group_of = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise RuntimeError("FusedAdam: fp32 contiguous CUDA parameters only")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                self._group_of[p] = group

    @torch.no_grad()
    def update_range(self, p, lo, hi, grad_scale=1.0):
        """Adam on elements [lo, hi) of p (its gradient scaled by grad_scale)."""
        if hi <= lo or p not in self._group_of:
            return
        group, st = self._group_of[p], self.state[p]
        b1, b2 = group["betas"]
        g = p.grad
        if not g.is_contiguous():
            raise RuntimeError("FusedAdam: contiguous gradients only")
        mirror = getattr(p, "_rn_f16", None)     # f16 copy kept by HashGridEncoding
        f4, f2 = 4 * lo, 2 * lo
        lib().adam(p.data_ptr() + f4, g.data_ptr() + f4, st["exp_avg"].data_ptr() + f4,
                   st["exp_avg_sq"].data_ptr() + f4, hi - lo, float(group["lr"]), float(b1),
                   float(b2), float(group["eps"]), int(st["step"]), float(grad_scale),
                   None if mirror is None else mirror.data_ptr() + f2,
                   0 if mirror is None else hi - lo,
                   torch.cuda.current_stream(p.device).cuda_stream)

    @torch.no_grad()
    def end_step(self):
        for p in self._group_of:
            # the kernel wrote p in place behind autograd's back: bump the
            # epoch the modules' derived caches (f16 fragments) key on; the
            # f16 table mirror was refreshed by the same pass
            p._rn_epoch = getattr(p, "_rn_epoch", 0) + 1
            if getattr(p, "_rn_f16", None) is not None:
                p._rn_f16_key = (p._version, p._rn_epoch)
        self._group_of = {}
