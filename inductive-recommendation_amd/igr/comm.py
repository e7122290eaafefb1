"""igr.comm - the collectives of the sharded path (igr.dist, igr.dist_train).

One place for the two exchange patterns the path has: the all-reduce (sum) of
partial item rows and the all-gather of batch ids / bitmaps.  On RCCL
(backend 'nccl') device tensors go to the collective as they are.  On gloo
(CPU tests and one-GPU rehearsals, where several ranks may share a device) a
device tensor is staged through host memory with synchronous copies: gloo is
only ever handed CPU tensors.
"""
import torch
import torch.distributed as dist


class _Done:
    """A collective that has already completed (the staged gloo path is synchronous)."""

    def wait(self):
        return True


def _staged(t, group):
    return t.is_cuda and dist.get_backend(group) == 'gloo'


def all_reduce_sum(t, group=None, async_op=False):
    """t = sum over ranks of t, in place; returns a work handle when async_op."""
    if _staged(t, group):
        host = t.detach().to('cpu', copy=True)  # synchronous device -> host copy
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        t.copy_(host)  # host -> device on the current stream, ordered before later kernels
        return _Done() if async_op else None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def all_gather_into(out, t, group=None):
    """out = the ranks' t, concatenated in rank order along the first dimension."""
    if _staged(t, group):
        host = t.detach().to('cpu', copy=True).contiguous()
        host_out = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(host_out, host, group=group)
        out.copy_(host_out)
        return out
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def all_reduce_sum_host(a, group=None, device=None):
    """numpy int64 / float array -> its sum over ranks (set-up data that lives on the
    host).  gloo reduces it where it is; RCCL reduces device tensors, so the array
    makes a round trip through `device`."""
    import numpy as np
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dist.get_backend(group) == 'gloo':
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t.numpy()
    td = t.to(device)
    dist.all_reduce(td, op=dist.ReduceOp.SUM, group=group)
    return td.cpu().numpy()
