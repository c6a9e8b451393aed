"""Minibatch pipeline of the demos: the replacement for

    dataset = tf.data.Dataset.from_tensor_slices((Xtrain, Ytrain))
    dataset = dataset.shuffle(buffer_size=num_data, seed=seed)
    dataset = dataset.batch(num_minibatch).repeat()
    train_iter = iter(dataset)                      # demos/demo_tf2.py:51-56

with the same pipeline semantics: `shuffle` draws from a buffer of
`buffer_size` elements and, by default, reshuffles on every pass
(reshuffle_each_iteration=True); `batch` emits the remainder as a short final
batch unless drop_remainder; `repeat()` without a count cycles forever and
applies to everything before it, so each epoch is a fresh shuffle.  The
stream is seeded (numpy PCG64) but is not TF's random stream: the element
order differs from TF's, the distribution does not.

The arrays stay where they are: device tensors are batched by an on-device
gather (one index_select per component), numpy arrays by numpy indexing, so a
training loop over HBM-resident data does no host round trip per step.
"""
import numpy as np
import torch


class Dataset:
    """tf.data.Dataset subset: from_tensor_slices / shuffle / batch / repeat / take."""

    def __init__(self, tensors, ops=()):
        self._tensors = tensors
        self._ops = tuple(ops)
        n = {len(t) for t in tensors}
        if len(n) != 1:
            raise ValueError("all components need the same leading dimension")
        self._n = n.pop()

    @classmethod
    def from_tensor_slices(cls, tensors):
        if not isinstance(tensors, (tuple, list)):
            tensors = (tensors,)
        return cls(tuple(tensors))

    def _with(self, op):
        return Dataset(self._tensors, self._ops + (op,))

    def shuffle(self, buffer_size, seed=None, reshuffle_each_iteration=True):
        if buffer_size < 1:
            raise ValueError("buffer_size must be >= 1")
        return self._with(("shuffle", int(buffer_size), seed, bool(reshuffle_each_iteration)))

    def batch(self, batch_size, drop_remainder=False):
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        return self._with(("batch", int(batch_size), bool(drop_remainder)))

    def repeat(self, count=None):
        return self._with(("repeat", count))

    def take(self, count):
        return self._with(("take", int(count)))

    # -------------------------------------------------------------------- iteration
    def _epoch_order(self, shuffle, rng):
        """Element order of one pass: a buffered shuffle (uniform permutation when
        the buffer holds the whole dataset)."""
        n = self._n
        if shuffle is None:
            return np.arange(n)
        buf_size = shuffle[1]
        if buf_size >= n:
            return rng.permutation(n)
        order = np.empty(n, np.int64)
        buf = list(range(min(buf_size, n)))
        nxt = len(buf)
        for i in range(n):
            j = int(rng.integers(len(buf)))
            order[i] = buf[j]
            if nxt < n:
                buf[j] = nxt
                nxt += 1
            else:
                buf[j] = buf[-1]
                buf.pop()
        return order

    def _gather(self, idx):
        out = []
        for t in self._tensors:
            if isinstance(t, torch.Tensor):
                out.append(t.index_select(0, torch.as_tensor(idx, device=t.device)))
            else:
                out.append(np.asarray(t)[idx])
        return tuple(out)

    def __iter__(self):
        shuffle = batch = None
        repeat = 1
        take = None
        for op in self._ops:
            if op[0] == "shuffle":
                shuffle = op
            elif op[0] == "batch":
                batch = op
            elif op[0] == "repeat":
                repeat = op[1]
            elif op[0] == "take":
                take = op[1]
        rng = np.random.default_rng(shuffle[2] if shuffle is not None else None)
        order0 = None
        emitted = 0
        epoch = 0
        while repeat is None or epoch < repeat:
            if shuffle is not None and (shuffle[3] or order0 is None):
                order = self._epoch_order(shuffle, rng)
                order0 = order
            else:
                order = order0 if order0 is not None else self._epoch_order(None, rng)
            step = batch[1] if batch is not None else 1
            for s in range(0, self._n, step):
                idx = order[s:s + step]
                if batch is not None and batch[2] and len(idx) < step:
                    break
                if take is not None and emitted >= take:
                    return
                items = self._gather(idx)
                if batch is None:
                    items = tuple(x[0] for x in items)
                yield items if len(items) > 1 else items[0]
                emitted += 1
            epoch += 1
