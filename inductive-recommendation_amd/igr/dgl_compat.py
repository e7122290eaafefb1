"""igr.dgl_compat - the slice of the DGL API the reference calls, backed by igr.

The reference reaches its graph arithmetic through exactly two DGL entry points
(`import dgl`, model.py:11):

    g = dgl.graph((column, row), num_nodes=n, device=dev)          model.py:103-105, 4183, 4194, 4035
    dgl.ops.gspmm(g, 'mul', 'sum', lhs_data=X, rhs_data=vals)       model.py:106, 4184, 4196, 4037
    dgl.ops.gspmm(g, 'copy_rhs', 'max' | 'sum', lhs_data=None, rhs_data=alpha)   model.py:4270, 4273

so replacing that import with `import igr.dgl_compat as dgl` moves those call
sites onto the HIP kernels with no other edit: same argument names, same
autograd behaviour (gradients with respect to lhs_data and rhs_data; the max
reduction sends each row's gradient to its arg-max edge, as DGL's does), errors
raised as exceptions.  `gsddmm(g, 'dot', lhs, rhs, h)` is offered beside them for
the masked per-edge dot product the reference writes by hand (model.py:4246-4255).
"""
import types

from . import ops as _ops

graph = _ops.graph
ops = types.SimpleNamespace(gspmm=_ops.gspmm, gsddmm=_ops.gsddmm)
DGLError = _ops.IgrError
