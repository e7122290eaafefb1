"""igr.optim - fused Adam on the HIP kernel (igr_adam_f32).

Drop-in for the `Adam` the reference resolves by name (trainer.py:44-46):
same constructor (params, lr, betas, eps, weight_decay) and torch.optim.Adam
update rule, one pass over (param, grad, exp_avg, exp_avg_sq) per tensor
instead of torch's multi-kernel foreach sequence.
"""
import ctypes

import torch

from . import _lib as L

# tensors up to this many elements share one launch (igr_adam_multi_f32); larger ones take
# igr_adam_f32, whose non-temporal traffic pays on tables that do not fit the caches
SMALL_NUMEL = 1 << 18


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError('invalid Adam hyper-parameters')
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.device_step = None  # (counter, base): step = state step + 1 + *counter, read on the device

    def set_device_step(self, counter):
        """hipGraph mode: the kernel adds *counter (device int64, the replays so far)
        to each tensor's step at the time of this call; the host counts stay put
        until advance_host_steps().  None returns to host-counted steps."""
        self.device_step = counter

    def advance_host_steps(self, n):
        for group in self.param_groups:
            for p in group['params']:
                st = self.state.get(p)
                if st:
                    st['step'] += n

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        ctr = self.device_step
        ctr_p = ctypes.c_void_p(0 if ctr is None else ctr.data_ptr())
        for group in self.param_groups:
            b1, b2 = group['betas']
            hyper = (float(group['lr']), float(b1), float(b2), float(group['eps']), float(group['weight_decay']))
            small = []  # (param, grad, state): tensors that share one launch (igr_adam_multi_f32)
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError('igr Adam does not support sparse gradients')
                if not p.is_cuda:
                    raise L.IgrError('igr Adam needs parameters on a ROCm device (no CPU fallback)')
                st = self.state[p]
                if not st:
                    st['step'] = 0
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                if ctr is None:
                    st['step'] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                assert p.is_contiguous() and p.dtype == torch.float32
                step = st['step'] if ctr is None else st['step'] + 1
                if p.numel() <= SMALL_NUMEL and all(t.data_ptr() % 16 == 0 for t in (p, g, st['exp_avg'],
                                                                                      st['exp_avg_sq'])):
                    small.append((p, g, st, step))
                    continue
                L.call('igr_adam_f32', p.numel(), ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                       ctypes.c_void_p(st['exp_avg'].data_ptr()), ctypes.c_void_p(st['exp_avg_sq'].data_ptr()),
                       *hyper, step, ctr_p, stream)
            for i in range(0, len(small), L.ADAM_MAX_SLOTS):
                chunk = small[i:i + L.ADAM_MAX_SLOTS]
                slots = (L.IgrAdamSlot * len(chunk))()
                for s, (p, g, st, step) in zip(slots, chunk):
                    s.param, s.grad = p.data_ptr(), g.data_ptr()
                    s.exp_avg, s.exp_avg_sq = st['exp_avg'].data_ptr(), st['exp_avg_sq'].data_ptr()
                    s.n, s.step = p.numel(), step
                L.call('igr_adam_multi_f32', len(chunk), ctypes.cast(slots, ctypes.c_void_p), *hyper, ctr_p, stream)
        return loss
