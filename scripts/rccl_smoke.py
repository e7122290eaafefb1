"""RCCL plumbing check on however many GPUs the box has (one is enough): the
process group bench.py creates (default stream priority), an async all-reduce
of a slice overlapped with a SpMM on the compute stream, and the float64 MAX
reduce bench.py ends with.  Run under torch.distributed.run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev)
    from igr.dist import BipartiteShard
    rng = np.random.default_rng(0)
    U, I = 20000, 3000
    pairs = np.stack([rng.integers(0, U, 200000), rng.integers(0, I, 200000)], 1)
    sh = BipartiteShard(pairs, U, I, rank, world, dev, item_chunks=4)
    xu = torch.randn(sh.u1 - sh.u0, 64, device=dev)
    xi = torch.randn(I, 64, device=dev)
    yu, yi = sh.layer(xu, xi)
    ref = yi.clone()
    # the layer's exchange pattern explicitly (at world 1 layer() issues none):
    # async all-reduces of row slices, then the compute stream waits on them
    works = [dist.all_reduce(yi[r0:r1], op=dist.ReduceOp.SUM, async_op=True) for r0, r1, _ in sh.chunks]
    yu2 = torch.empty_like(yu)
    from igr import ops
    ops.spmm(sh.user_block, xi, sh.user_vals, out=yu2)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    assert torch.equal(yi, ref * world) or world > 1, 'all-reduce at world 1 must be the identity'
    assert torch.equal(yu2, yu)
    t = torch.tensor([float(rank)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    print(f'rank {rank}/{world}: layer ok, |y_items| {float(yi.abs().sum()):.4f}, max rank {float(t)}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
