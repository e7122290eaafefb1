"""igr.trainer - the reference's trainer surface (trainer.py) for the path.

BasicTrainer.train / eval / calculate_metrics keep the reference's loop,
early stopping on NDCG@topks[4], checkpoint naming and metric definitions
(trainer.py:25-210).  BPRTrainer and IGCNTrainer keep the per-batch loss
math (trainer.py:403-429, 518-561); by default the loss terms go through the
fused HIP BPR kernel (model.bpr_loss / aux_loss), and `fused: False` in the
trainer config runs the reference's exact op sequence on bpr_forward.
Evaluation computes the representation once per eval instead of once per
512-user batch (the reference's predict re-propagates, model.py:123); in
eval mode both are the same function of the weights.

Trainer config extensions (all optional): 'sampler': 'device' (default, HIP
sampler, igr.sampler) or 'host' (vectorised numpy); 'fused' (default True);
'seed'; 'graph' (default 'auto'): train_one_epoch replays one hipGraph-captured
step (StepGraph) instead of issuing every launch from Python.  'auto' takes the
captured step where it is proven bitwise equal to eager steps (graph_mode_for:
device sampler, fused losses, a model whose dropout masks come from device
counters, an unsharded trainer on a ROCm device); True insists on it wherever the
device sampler runs, False always steps eagerly.  The epoch loss is accumulated
on the device and read once per epoch (the reference syncs with loss.item()
every step, trainer.py:556).
"""
import contextlib
import ctypes
import itertools
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F
from torch.optim import SGD  # noqa: F401  (resolved by name, trainer.py:44-46)
from torch.optim import Adam as TorchAdam  # noqa: F401

from . import _lib as L
from . import ops
from .dataset import AuxiliaryDataset, BPRBatchSampler
from .model import batch_rep_pays
from .optim import Adam  # noqa: F401  fused HIP Adam, resolved by name 'Adam'
from .sampler import DeviceBPRSampler


def get_trainer(config, dataset, model):
    """trainer.py:16-22."""
    config = config.copy()
    config['dataset'] = dataset
    config['model'] = model
    trainer = getattr(sys.modules[__name__], config['name'])
    return trainer(config)


def eval_keys(eval_data, n_users, n_items):
    """The eval lists as sorted (user * n_items + item) keys plus their lengths:
    what calculate_metrics matches the ranking against (reusable across evals)."""
    ptr, flat = _csr(eval_data, n_users)
    lens = np.diff(ptr).astype(np.int32)
    return np.unique(np.repeat(np.arange(n_users, dtype=np.int64), lens) * n_items + flat), lens


def calculate_metrics(eval_data, rec_items, topks, keys=None):
    """trainer.py:115-144, vectorised: Precision/Recall/NDCG@k averaged over
    users with a non-empty eval set.  keys: eval_keys(eval_data, ...) computed
    once (with n_items >= every item id in eval_data and rec_items)."""
    n_users, kmax = rec_items.shape
    if keys is None:
        n_items = int(max(rec_items.max(initial=0),
                          max((max(x) for x in eval_data[:n_users] if x), default=0)) + 1)
        keys = eval_keys(eval_data, n_users, n_items) + (n_items,)
    ev_keys, lens, n_items = keys
    rk = (np.arange(n_users, dtype=np.int64)[:, None] * n_items + rec_items).ravel()
    j = np.minimum(np.searchsorted(ev_keys, rk), max(len(ev_keys) - 1, 0))
    hit = (ev_keys[j] == rk).reshape(n_users, kmax).astype(np.float32) if len(ev_keys) else \
        np.zeros((n_users, kmax), np.float32)
    res = {'Precision': {}, 'Recall': {}, 'NDCG': {}}
    for k in topks:
        hit_num = hit[:, :k].sum(1)
        with np.errstate(invalid='ignore', divide='ignore'):
            recalls = hit_num / lens
        max_hit = np.minimum(lens, k)
        max_hit_matrix = (np.arange(k)[None, :] < max_hit[:, None]).astype(np.float32)
        den = np.log2(np.arange(2, k + 2, dtype=np.float32))[None, :]
        dcg = (hit[:, :k] / den).sum(1)
        idcg = (max_hit_matrix / den).sum(1)
        with np.errstate(invalid='ignore', divide='ignore'):
            ndcg = dcg / idcg
        m = max_hit > 0
        res['Precision'][k] = (hit_num / k)[m].mean()
        res['Recall'][k] = recalls[m].mean()
        res['NDCG'][k] = ndcg[m].mean()
    return res


def calculate_metrics_device(ev_keys, lens, rec, topks, n_items):
    """calculate_metrics (trainer.py:115-144) on the device: `rec` the [users, kmax] int64
    ranking as the top-k kernel left it, `ev_keys` the sorted (user * n_items + item) keys
    of the eval lists, `lens` their lengths.  Hits by one searchsorted; hit counts, DCG and
    ideal DCG for every k from prefix sums along the ranking; the averages over users with a
    non-empty list in float64.  One small copy to the host at the end (no sync before it)."""
    n_users, kmax = rec.shape
    dev = rec.device
    rk = (torch.arange(n_users, device=dev, dtype=torch.int64)[:, None] * n_items + rec).reshape(-1)
    if ev_keys.numel():
        j = torch.searchsorted(ev_keys, rk).clamp_(max=ev_keys.numel() - 1)
        hit = (ev_keys[j] == rk).view(n_users, kmax).to(torch.float32)
    else:
        hit = torch.zeros(n_users, kmax, dtype=torch.float32, device=dev)
    # the reference's float32 discounts, computed by the same numpy call
    den = torch.from_numpy(np.log2(np.arange(2, kmax + 2, dtype=np.float32))).to(dev)
    ks = torch.tensor(list(topks), dtype=torch.int64, device=dev)
    hit_num = torch.cumsum(hit, 1)[:, ks - 1]                       # [users, n_k]
    dcg = torch.cumsum(hit / den, 1)[:, ks - 1]
    lens_f = lens.to(torch.float32)
    max_hit = torch.minimum(lens.to(torch.int64)[:, None], ks[None, :])
    ideal = torch.cumsum(1. / den, 0)
    idcg = ideal[(max_hit - 1).clamp_(min=0)]
    live = (lens > 0)
    n_live = live.sum().to(torch.float64)
    mask = live[:, None].to(torch.float64)

    def avg(x):  # mean over the users with a non-empty eval list
        return (x.to(torch.float64) * mask).sum(0) / n_live
    safe_len = torch.where(live, lens_f, torch.ones((), device=dev))[:, None]
    out = torch.stack([avg(hit_num / ks[None, :].to(torch.float32)), avg(hit_num / safe_len), avg(dcg / idcg)]).cpu().numpy()
    res = {'Precision': {}, 'Recall': {}, 'NDCG': {}}
    for c, k in enumerate(topks):
        res['Precision'][k], res['Recall'][k], res['NDCG'][k] = out[0, c], out[1, c], out[2, c]
    return res


def _csr(lists, n):
    """Per-user lists as (row_ptr, flat items); the iteration runs in C (map / chain)."""
    lists = lists[:n]
    lens = np.fromiter(map(len, lists), dtype=np.int64, count=len(lists))
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    flat = np.fromiter(itertools.chain.from_iterable(lists), dtype=np.int64, count=int(ptr[-1]))
    return ptr, flat


def _csr_concat(a, b):
    """Row-wise concatenation of two CSRs over the same rows: row u = a's items, then b's."""
    (pa, fa), (pb, fb) = a, b
    ptr = pa + pb
    flat = np.empty(len(fa) + len(fb), dtype=np.int64)
    la, lb = np.diff(pa), np.diff(pb)
    flat[np.arange(len(fa)) + np.repeat(pb[:-1], la)] = fa
    flat[np.arange(len(fb)) + np.repeat(pa[1:], lb)] = fb
    return ptr, flat


class BasicTrainer:
    """trainer.py:25-253."""

    def __init__(self, trainer_config):
        self.config = trainer_config
        self.name = trainer_config['name']
        self.dataset = trainer_config['dataset']
        self.model = trainer_config['model']
        self.topks = trainer_config['topks']
        self.device = trainer_config['device']
        self.n_epochs = trainer_config['n_epochs']
        self.max_patience = trainer_config.get('max_patience', 50)
        self.val_interval = trainer_config.get('val_interval', 1)
        self.test_batch_size = trainer_config['test_batch_size']
        self.epoch = 0
        self.best_ndcg = -np.inf
        self.save_path = None
        self.opt = None
        self.verbose = trainer_config.get('verbose', True)
        # True while train() runs (or when the caller vouches that train / val / test lists stay
        # as they are): eval() then reuses the exclusion CSR and the metric keys between calls
        self.static_eval_lists = trainer_config.get('static_eval_lists', False)

    def initialize_optimizer(self):
        opt = getattr(sys.modules[__name__], self.config['optimizer'])
        self.opt = opt(self.model.parameters(), lr=self.config['lr'])

    def train_one_epoch(self):
        raise NotImplementedError

    def record(self, writer, stage, metrics):
        """trainer.py:49-56: every metric@k of one eval to a tensorboard-style writer."""
        for metric in metrics:
            for k in self.topks:
                writer.add_scalar('{:s}_{:s}/{:s}_{:s}@{:d}'.format(self.model.name, self.name, stage, metric, k),
                                  metrics[metric][k], self.epoch)

    def train(self, verbose=True, writer=None):
        """trainer.py:58-113."""
        if not self.model.trainable:
            _, metrics, _ = self.eval('val')
            return metrics['NDCG'][self.topks[5]]
        ckpt_dir = self.config.get('checkpoint_dir', 'checkpoints')
        os.makedirs(ckpt_dir, exist_ok=True)
        static, self.static_eval_lists = self.static_eval_lists, True  # nothing edits the lists in here
        try:
            self._epochs(verbose, writer, ckpt_dir)
        finally:
            self.static_eval_lists = static
            if not static:
                self.__dict__.pop('_excl', None)
                self.__dict__.pop('_eval_keys', None)
                self.__dict__.pop('_eval_keys_dev', None)
        self._close_step_graph()  # load() below rebuilds graph structures a captured step points at
        if self.save_path:
            self.model.load(self.save_path)
        return self.best_ndcg

    def _epochs(self, verbose, writer, ckpt_dir):
        """The epoch loop of train(): trainer.py:69-110."""
        patience = self.max_patience
        for self.epoch in range(self.n_epochs):
            start = time.time()
            self.model.train()
            loss = self.train_one_epoch()
            _, metrics, _ = self.eval('train')
            if verbose:
                print('Epoch {:d}/{:d}, Loss: {:.6f}, Time: {:.3f}s'.format(self.epoch, self.n_epochs, loss,
                                                                          time.time() - start))
            if writer:
                writer.add_scalar('{:s}_{:s}/train_loss'.format(self.model.name, self.name), loss, self.epoch)
                self.record(writer, 'train', metrics)
            if (self.epoch + 1) % self.val_interval != 0:
                continue
            start = time.time()
            results, metrics, _ = self.eval('val')
            if verbose:
                print('Validation result. {:s}Time: {:.3f}s'.format(results, time.time() - start))
            if writer:
                self.record(writer, 'validation', metrics)
            ndcg = metrics['NDCG'][self.topks[4]]
            if ndcg > self.best_ndcg:
                if self.save_path and os.path.exists(self.save_path):
                    os.remove(self.save_path)
                self.save_path = os.path.join(ckpt_dir, '{:s}_{:s}_{:s}_{:.3f}.pth'.format(
                    self.model.name, self.name, self.dataset.name, ndcg * 100))
                self.best_ndcg = ndcg
                self.model.save(self.save_path)
                patience = self.max_patience
                if verbose:
                    print('Best NDCG, save model to {:s}'.format(self.save_path))
            else:
                patience -= self.val_interval
                if patience <= 0:
                    if verbose:
                        print('Early stopping!')
                    break

    def _close_step_graph(self):
        sg = getattr(self, '_step_graph', None)
        if sg is not None:
            sg.close()
            self._step_graph = None

    def _graph_epoch(self):
        """The epoch through a StepGraph when graph_mode_for(self) says so; None = run it
        eagerly (leaving graph mode first)."""
        if graph_mode_for(self):
            return graph_epoch(self)
        self._close_step_graph()
        return None

    def _eager_step_guard(self):
        """A step() called from outside while a captured step is live (its counters are on
        the device): hand the counters back to the host first, so eager and captured steps
        can be mixed freely."""
        if getattr(self, '_step_graph', None) is not None and not getattr(self, '_in_graph_body', False):
            self._close_step_graph()

    def calculate_metrics(self, eval_data, rec_items):
        n_items = max(int(self.dataset.n_items), int(rec_items.max(initial=0)) + 1)
        if not self.static_eval_lists:
            return calculate_metrics(eval_data, rec_items, self.topks,
                                     keys=eval_keys(eval_data, rec_items.shape[0], n_items) + (n_items,))
        # inside train() the eval lists do not change: their keys are built once (the entry
        # holds the list object, so its id cannot pass to another list)
        cache = self.__dict__.setdefault('_eval_keys', {})
        key = (id(eval_data), len(eval_data), rec_items.shape[0], n_items)
        if key not in cache:
            cache[key] = (eval_data, eval_keys(eval_data, rec_items.shape[0], n_items) + (n_items,))
        return calculate_metrics(eval_data, rec_items, self.topks, keys=cache[key][1])

    def _calculate_metrics_device(self, eval_data, rec):
        n_items = int(self.dataset.n_items)
        cache = self.__dict__.setdefault('_eval_keys_dev', {}) if self.static_eval_lists else {}
        key = (id(eval_data), len(eval_data), rec.shape[0], n_items)
        if key not in cache:
            keys, lens = eval_keys(eval_data, rec.shape[0], n_items)
            cache[key] = (eval_data, torch.from_numpy(keys).to(rec.device), torch.from_numpy(lens).to(rec.device))
        _, keys, lens = cache[key]
        return calculate_metrics_device(keys, lens, rec, self.topks, n_items)

    @torch.no_grad()
    def rank(self, val_or_test, banned_items=None, to_host=True):
        """Top-max(topks) items per user, train items (and val items for
        'test') excluded except for split 'train' (trainer.py:146-170).
        One propagation per eval; per user batch: MFMA score GEMM,
        igr_mask_scores (the exclusion CSR is uploaded once, each batch passes
        its slice of row_ptr) and igr_topk (value desc, ties by index asc)."""
        self.model.eval()
        n_users = self.dataset.n_users
        rep = self.model.get_rep()
        excl = None
        if val_or_test != 'train':
            # inside train() the exclusion lists do not change: one device CSR per split,
            # otherwise rebuilt from the lists at every call, as the reference reads them
            cache = self.__dict__.setdefault('_excl', {}) if self.static_eval_lists else {}
            ck = (val_or_test, id(self.dataset.train_data), id(self.dataset.val_data), n_users)
            if ck not in cache:
                ptr, flat = _csr(self.dataset.train_data, n_users)
                if val_or_test == 'test':
                    ptr, flat = _csr_concat((ptr, flat), _csr(self.dataset.val_data, n_users))
                cache[ck] = (torch.from_numpy(ptr.astype(np.int64)).to(self.device),
                             torch.from_numpy(flat.astype(np.int32)).to(self.device),
                             self.dataset.train_data, self.dataset.val_data)
            excl = cache[ck]
        kmax = max(self.topks)
        rec = []
        # test_batch_size bounds the reference's score matrix; rows are ranked
        # independently, so a batch sized for HBM (~1 GB of scores) gives the same
        # result with enough rows to fill the chip (measured on MI355X, Gowalla
        # shape: 512 -> 4096 users per batch halves the eval)
        batch = max(self.test_batch_size, (1 << 28) // max(1, self.dataset.n_items))
        for s in range(0, n_users, batch):
            e = min(n_users, s + batch)
            users = torch.arange(s, e, dtype=torch.int64, device=self.device)
            scores = self.model.predict(users, rep)
            if excl is not None:
                ops.mask_scores(scores, excl[0][s:e + 1], excl[1])
            if banned_items is not None:
                scores[:, torch.as_tensor(banned_items, device=self.device)] = -np.inf
            _, items = ops.topk(scores, kmax, values=False)
            rec.append(items)  # stays on the device: one copy (and sync) per eval, not per batch
        rec = torch.cat(rec)
        return rec.cpu().numpy() if to_host else rec

    def eval(self, val_or_test, banned_items=None):
        """trainer.py:146-210; returns the reference's triple (result string,
        metrics, prot_results), the last one the empty list it is there (184-210).

        The reference iterates its test_user_loader (a torch DataLoader,
        trainer.py:41-42, 151), and creating a DataLoader iterator draws one
        int64 base seed from the global CPU generator.  The same draw is made
        here, so a seeded run stays on the reference's CPU random stream (the
        dropout masks of dropout_rng='cpu' and anything seeded after an eval)."""
        torch.empty((), dtype=torch.int64).random_()
        eval_data = getattr(self.dataset, val_or_test + '_data')
        if torch.device(self.device).type == 'cuda':
            # the ranking stays on the device and the metrics are computed there
            rec_items = self.rank(val_or_test, banned_items, to_host=False)
            metrics = self._calculate_metrics_device(eval_data, rec_items)
        else:
            rec_items = self.rank(val_or_test, banned_items)
            metrics = self.calculate_metrics(eval_data, rec_items)
        fmt = lambda m: ''.join('{:.3f}, '.format(metrics[m][k] * 100.) for k in self.topks)  # noqa: E731
        results = 'Precision: {:s}Recall: {:s}NDCG: {:s}'.format(fmt('Precision'), fmt('Recall'), fmt('NDCG'))
        return results, metrics, []

    def inductive_eval(self, n_old_users, n_old_items):
        """trainer.py:212-253: the test metrics of a model moved to a grown dataset,
        over six slices - all / old / new users on all items, all users on old /
        new items (the other items banned from the ranking), old users on old
        items.  Prints the reference's six lines; also returns the metrics by
        slice (the reference returns nothing).  dataset.test_data is left as found."""
        ds = self.dataset
        full = ds.test_data
        n_users, n_items = ds.n_users, ds.n_items
        old_items = lambda u: [i for i in full[u] if i < n_old_items]  # noqa: E731
        new_items = lambda u: [i for i in full[u] if i >= n_old_items]  # noqa: E731
        ban_new = np.arange(n_old_items, n_items)
        ban_old = np.arange(n_old_items)
        slices = [
            ('All users and all items', lambda u: full[u], None),
            ('Old users and all items', lambda u: full[u] if u < n_old_users else [], None),
            ('New users and all items', lambda u: full[u] if u >= n_old_users else [], None),
            ('All users and old items', old_items, ban_new),
            ('All users and new items', new_items, ban_old),
            ('Old users and old items', lambda u: old_items(u) if u < n_old_users else [], ban_new),
        ]
        out = {}
        try:
            for name, pick, banned in slices:
                ds.test_data = [list(pick(u)) for u in range(n_users)]
                results, metrics, _ = self.eval('test', banned_items=banned)
                print('{:s} result. {:s}'.format(name, results))
                out[name] = metrics
        finally:
            ds.test_data = full
        return out


class StepGraph:
    """One whole training step - device BPR sampling (main + aux batch), the
    forward, the backward and the fused Adam - captured once in a hipGraph and
    replayed (the "graph" trainer option).  On graphs the size of ML-1M a step
    is ~100 short launches whose host-side cost (autograd, ctypes) exceeds the
    GPU time; a replay issues them with no host work at all.

    Everything that changes from step to step lives on the device: the step
    counter `ctr` (replays so far) is added on the device to the sampler's
    counter offset, the dropout-mask offset and Adam's step; the loss is summed
    into a device scalar; the feature values are updated in place on anneal.
    So a replay is the same computation as an eager step at the same counters.
    The host counters are brought forward in close()."""

    def __init__(self, trainer, batch_size, warmup=2):
        self.tr, self.B = trainer, int(batch_size)
        model, dev = trainer.model, trainer.sampler.device
        self.ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self.aux = getattr(trainer, 'aux_sampler', None)
        self.s0 = trainer.sampler.step
        self.a0 = self.aux.step if self.aux is not None else 0
        self.d0 = getattr(model, '_drop_step', -1)
        self.n = 0  # real steps run in graph mode (warm-up + replays + eager tails)
        # the replay reads these objects' device arrays: keep them alive while the graph exists
        self._keep = [getattr(model, a, None) for a in ('norm_adj', 'norm_vals', 'feat_mat', 'feat_base', 'row_sum')]
        trainer.opt.set_device_step(self.ctr)
        model.device_step = self.ctr
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # allocations and lazy state outside the capture
            for _ in range(warmup):
                self.body(self.B)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.body(self.B, count=False)

    def _draw_stream(self, n):
        """The stream the batches are drawn on, or None for the current one.  With the fused
        full-graph step the propagation does not read the batch: drawn on a second stream
        (the aux term's, inside a capture) the sampling runs beside it, and the model joins
        that stream just before the batch's first use (BasicModel._join_batch_stream).  The
        batch-row step reads the batch first; other trainers never join."""
        tr, model = self.tr, self.tr.model
        if not getattr(tr, 'fused', False) or not hasattr(model, 'bpr_loss') or \
                not hasattr(model, '_join_batch_stream') or model.config.get('draw_stream', True) is False:
            return None
        rows = model._rows_path(n) if hasattr(model, '_rows_path') else batch_rep_pays(model, n)
        if rows:
            return None
        # only the stream the step forks anyway (the aux term's, inside a capture): a fork and a join
        # made for the sampling alone cost more than the kernel they hide (LightGCN at the ML-1M
        # shape: 0.19 -> 0.22 ms; IGCN, whose aux term already runs there: 0.32 -> 0.30 ms)
        return model._aux_stream() if hasattr(model, '_aux_stream') else None

    def body(self, n, count=True):
        tr = self.tr
        side = self._draw_stream(n)
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
            tr.model._batch_stream = side
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            u, p, ng = tr.sampler.sample(n, offset=self.s0, offset_dev=self.ctr)
            if self.aux is not None:
                au, ap, an = self.aux.sample(n, offset=self.a0, offset_dev=self.ctr)
        tr._in_graph_body = True
        try:
            if self.aux is not None:
                _summed_step(tr, self.loss_sum, n, u, p, ng, au, ap, an)
            else:
                _summed_step(tr, self.loss_sum, n, u, p, ng)
        finally:
            tr._in_graph_body = False
        tr.model.__dict__.pop('_batch_stream', None)  # consumed by the model; never left behind
        L.call('igr_counter_add', ctypes.c_void_p(self.ctr.data_ptr()), 1, ops._stream())
        if count:
            self.n += 1

    def replay(self):
        self.graph.replay()
        self.n += 1

    def take_loss(self):
        """Sum of loss * batch over the steps since the last call (one host sync)."""
        v = float(self.loss_sum)
        self.loss_sum.zero_()
        return v

    def close(self):
        """Back to eager steps: host counters advanced by the steps run here."""
        tr, model = self.tr, self.tr.model
        tr.sampler.step = self.s0 + self.n
        if self.aux is not None:
            self.aux.step = self.a0 + self.n
        if hasattr(model, '_drop_seed'):
            model._drop_step = self.d0 + self.n
        tr.opt.set_device_step(None)
        tr.opt.advance_host_steps(self.n)
        model.device_step = None
        self.graph = self._keep = None


def graph_mode_for(trainer):
    """Does train_one_epoch replay a captured step?  config['graph']: True / False, or 'auto'
    (the default): on exactly where the captured step has been shown bitwise equal to eager
    steps - the device sampler draws the batches, the losses are the fused ones, the model's
    dropout masks are counter-based (`graph_safe`: IGCN / IMF / AttIGCN / LightGCN unless
    dropout_rng = 'cpu'; NGCF and IMCGAE only at dropout 0, their node dropout draws from
    torch's generator), and the device is a GPU.  The sharded trainer (dist_train) has its own
    loop and never comes here."""
    want = trainer.config.get('graph', 'auto')
    if not isinstance(trainer.sampler, DeviceBPRSampler):
        return False  # host-drawn batches cannot be captured
    if want != 'auto':
        return bool(want)
    return bool(getattr(trainer, 'fused', False)) and bool(getattr(trainer.model, 'graph_safe', False)) and \
        hasattr(trainer.model, 'bpr_loss')


def graph_epoch(trainer):
    """train_one_epoch through a StepGraph: ceil(len / B) steps, the last one
    (a partial batch) run eagerly in the same device-counter mode."""
    B = trainer.config['batch_size']
    total = trainer.sampler.length
    full, tail = divmod(total, B)
    sg = getattr(trainer, '_step_graph', None)
    if sg is None:
        if full < 3:
            return None
        sg = trainer._step_graph = StepGraph(trainer, B)
        full -= 2  # the warm-up steps were real steps of this epoch
    for _ in range(full):
        sg.replay()
    if tail:
        sg.body(tail)
    return sg.take_loss() / total


def fused_loss_step(trainer, bpr, l2, aux=None):
    """loss = bpr + (l2_reg * l2 + aux_reg * aux), its backward and the optimizer
    step (trainer.py:551-555, 424-428) without scalar tensor arithmetic: the value
    comes from one kernel and the terms' gradients are the constant coefficients
    (cached device scalars handed to autograd).  Returns the detached loss."""
    c_l2 = float(trainer.l2_reg)
    c_aux = float(getattr(trainer, 'aux_reg', 0.0))
    acc = getattr(trainer, '_loss_acc', None)
    loss = ops.loss_combine(bpr, l2, aux, c_l2, c_aux, loss_sum=None if acc is None else acc[0],
                            weight=1.0 if acc is None else float(acc[1]))
    trainer._loss_acc = None  # consumed
    cache = trainer.__dict__.setdefault('_coef_cache', {})
    terms, grads = [], []
    for t, c in ((bpr, 1.0), (l2, c_l2), (aux, c_aux)):
        if t is None or not t.requires_grad or c == 0.0:  # a zero coefficient: exact-zero gradients
            continue
        if c not in cache:
            cache[c] = torch.tensor(c, dtype=torch.float32, device=t.device)
        terms.append(t)
        grads.append(cache[c])
    trainer.opt.zero_grad()
    scope = getattr(trainer.model, 'backward_scope', None)  # IGCN: the aux term's side stream
    with (scope() if scope is not None else contextlib.nullcontext()):
        torch.autograd.backward(terms, grads)
    trainer.opt.step()
    return loss


def _summed_step(trainer, total, n, *batch):
    """trainer.step(*batch) with total += loss * n on the device (inside the fused
    step's combine kernel when there is one); returns the loss."""
    trainer._loss_acc = (total, n)
    try:
        loss = trainer.step(*batch)
        if trainer._loss_acc is not None:  # not consumed: an unfused step
            total.add_(loss.detach() * n)
    finally:
        trainer._loss_acc = None
    return loss


def base_seed(trainer_config):
    """The trainer's sampling seed: config['seed'], or one drawn from torch's seed
    when the config has none (the reference's configs set none), so that the
    samplers of one trainer can be given distinct streams derived from it."""
    seed = trainer_config.get('seed')
    return int(torch.initial_seed() & 0x7fffffff) if seed is None else int(seed)


def make_sampler(trainer_config, dataset, seed):
    if trainer_config.get('sampler', 'device') == 'device' and torch.device(trainer_config['device']).type == 'cuda':
        return DeviceBPRSampler(dataset, trainer_config['batch_size'], trainer_config['device'], seed)
    return BPRBatchSampler(dataset, trainer_config['batch_size'], seed)


def _dev_batch(batch, device):
    return tuple(b if isinstance(b, torch.Tensor) else torch.from_numpy(b).to(device) for b in batch)


class BPRTrainer(BasicTrainer):
    """trainer.py:403-429."""

    def __init__(self, trainer_config):
        super().__init__(trainer_config)
        self.sampler = make_sampler(trainer_config, self.dataset, base_seed(trainer_config))
        self.initialize_optimizer()
        self.l2_reg = trainer_config['l2_reg']
        self.fused = trainer_config.get('fused', True)

    def step(self, users, pos_items, neg_items):
        """One training step on a device batch; returns the loss tensor."""
        self._eager_step_guard()
        if self.fused and hasattr(self.model, 'bpr_loss'):
            bpr_loss, l2 = self.model.bpr_loss(users, pos_items, neg_items, need_l2=self.l2_reg != 0)
            return fused_loss_step(self, bpr_loss, l2)
        else:
            users_r, pos_r, neg_r, l2_norm_sq = self.model.bpr_forward(users, pos_items, neg_items)
            pos_scores = torch.sum(users_r * pos_r, dim=1)
            neg_scores = torch.sum(users_r * neg_r, dim=1)
            loss = F.softplus(neg_scores - pos_scores).mean() + self.l2_reg * l2_norm_sq.mean()
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss

    def train_one_epoch(self):
        loss = self._graph_epoch()
        if loss is not None:
            return loss
        tot, cnt = torch.zeros((), dtype=torch.float32, device=self.device), 0
        for batch in self.sampler:
            u, p, n = _dev_batch(batch, self.device)
            _summed_step(self, tot, len(u), u, p, n)
            cnt += len(u)
        return float(tot) / cnt


class IGCNTrainer(BasicTrainer):
    """trainer.py:518-561: BPR on rep + l2 + aux BPR on the raw feature table (with w)."""

    def __init__(self, trainer_config):
        super().__init__(trainer_config)
        # two independent streams, as the reference's two DataLoaders (trainer.py:522-530):
        # with feature_ratio = 1 the aux dataset IS the dataset, so equal seeds would
        # train the aux term on exactly the main term's triples
        seed = base_seed(trainer_config)
        self.sampler = make_sampler(trainer_config, self.dataset, seed)
        self.aux_sampler = make_sampler(trainer_config,
                                        AuxiliaryDataset(self.dataset, self.model.user_map, self.model.item_map),
                                        seed + 1)
        self.initialize_optimizer()
        self.l2_reg = trainer_config['l2_reg']
        self.aux_reg = trainer_config['aux_reg']
        self.fused = trainer_config.get('fused', True)

    def step(self, users, pos_items, neg_items, a_users, a_pos, a_neg):
        self._eager_step_guard()
        m = self.model
        if self.fused:
            bpr_loss, l2, aux_loss = m.bpr_aux_loss(users, pos_items, neg_items, a_users, a_pos, a_neg,
                                                    need_l2=self.l2_reg != 0)
            return fused_loss_step(self, bpr_loss, l2, aux_loss)
        else:
            users_r, pos_r, neg_r, l2_norm_sq = m.bpr_forward(users, pos_items, neg_items)
            bpr_loss = F.softplus(torch.sum(users_r * neg_r, 1) - torch.sum(users_r * pos_r, 1)).mean()
            l2 = l2_norm_sq.mean()
            ue = m.embedding(a_users)
            pe = m.embedding(a_pos + len(m.user_map))
            ne = m.embedding(a_neg + len(m.user_map))
            aux_loss = F.softplus(torch.sum(ue * ne * m.w[None, :], 1) - torch.sum(ue * pe * m.w[None, :], 1)).mean()
        loss = bpr_loss + (self.l2_reg * l2 + self.aux_reg * aux_loss)
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss

    def train_one_epoch(self):
        loss = self._graph_epoch()
        if loss is not None:
            self.model.feat_mat_anneal()
            return loss
        tot, cnt = torch.zeros((), dtype=torch.float32, device=self.device), 0
        for main, aux in zip(self.sampler, self.aux_sampler):
            u, p, n = _dev_batch(main, self.device)
            au, ap, an = _dev_batch(aux, self.device)
            _summed_step(self, tot, len(au), u, p, n, au, ap, an)
            cnt += len(au)
        self.model.feat_mat_anneal()
        return float(tot) / cnt
