"""How well the sharded layer's stream structure hides an exchange that costs local memory
traffic (one GPU, no second device): rank 0 of an 8-way partition of the bench graph runs chained
layers (a) without any exchange and (b) with a stand-in exchange on a side stream that has the
stream semantics of an RCCL collective and, per item row chunk, copies the chunk back and forth
`--copies` times (device-local traffic of the order of a ring all-reduce's: 2 x (N-1)/N reads and
writes of the buffer).  It says nothing about xGMI; it shows whether side-stream work overlaps the
SpMM launches at all and what it costs them.  One JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--copies', type=int, default=2)
    ap.add_argument('--layers', type=int, default=40)
    ap.add_argument('--spin-cycles', type=int, default=0,
                    help='per chunk, also spin this many GPU cycles on the side stream (a collective that mostly '
                         'waits for remote data: time without memory traffic)')
    args = ap.parse_args()
    from igr import comm
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    from igr.graph import count_ids
    dev = torch.device('cuda')
    U, I, E, d, W = 10_000_000, 1_000_000, 200_000_000, 64, args.world
    su, si = synthetic_pairs(U, I, E, 0, stacked=False)
    total = np.concatenate([count_ids(su, U), count_ids(si, I)])
    e1 = E // W
    others = total - np.concatenate([count_ids(su[:e1], U), count_ids(si[:e1], I)])
    sh = BipartiteShard.from_stream(su, si, U, I, 0, W, dev, d=d, reduce=lambda c: c + others)
    del su, si
    g = torch.Generator(device=dev).manual_seed(0)
    xu = torch.randn(sh.u1 - sh.u0, d, generator=g, device=dev) * 0.1
    xi = torch.randn(I, d, generator=g, device=dev) * 0.1
    side = torch.cuda.Stream()
    tmp = torch.empty(I, d, device=dev)

    class Work:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    def standin(t, group=None, async_op=False):
        cur = torch.cuda.current_stream()
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(side):
            side.wait_event(ready)
            buf = tmp[:t.shape[0]]
            if args.spin_cycles:
                torch.cuda._sleep(args.spin_cycles)
            for _ in range(args.copies):
                buf.copy_(t)
                t.copy_(buf)
            done = torch.cuda.Event()
            done.record(side)
        w = Work(done)
        if not async_op:
            w.wait()
        return w

    def run(exchange):
        sh.exchange = exchange
        for _ in range(2):
            sh.propagate(xu, xi, 4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sh.propagate(xu, xi, args.layers)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.layers * 1e3
    plain = run(False)
    real = comm.all_reduce_sum
    comm.all_reduce_sum = standin
    try:
        with_x = run(True)
        # the exchange alone, nothing beside it
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            for r0, r1, _t in sh.chunks:
                standin(xi[r0:r1])
        torch.cuda.synchronize()
        alone = (time.perf_counter() - t0) / 10 * 1e3
    finally:
        comm.all_reduce_sum = real
    moved = args.copies * 2 * 2 * I * d * 4
    print(json.dumps({'world': W, 'rank': 0, 'local_nnz': sh.local_nnz, 'layer_ms_no_exchange': plain,
                      'layer_ms_with_standin_exchange': with_x, 'standin_exchange_alone_ms': alone,
                      'standin_bytes_per_layer': moved, 'spin_cycles_per_chunk': args.spin_cycles, 'hidden_fraction': 1.0 - max(0.0, with_x - plain) / alone}))


if __name__ == '__main__':
    main()
