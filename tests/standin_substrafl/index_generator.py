"""A seeded batch sampler with the attributes the torch algorithms read (the reference's
``BaseIndexGenerator`` contract: ``n_samples`` set once, ``num_updates`` draws per task,
``reset_counter`` / ``check_num_updates``), written for this stand-in."""

import numpy as np

from .exceptions import IndexGeneratorUpdateError


class NpIndexGenerator:
    def __init__(self, batch_size: int, num_updates: int, seed: int = 42):
        self._batch_size = batch_size
        self._num_updates = num_updates
        self._rng = np.random.default_rng(seed)
        self._n_samples = None
        self._pool = np.empty(0, dtype=np.int64)
        self._counter = 0

    @property
    def batch_size(self):
        return self._batch_size

    @property
    def num_updates(self):
        return self._num_updates

    @property
    def counter(self):
        return self._counter

    @property
    def n_samples(self):
        return self._n_samples

    @n_samples.setter
    def n_samples(self, n: int):
        self._n_samples = int(n)
        self._batch_size = min(self._batch_size, self._n_samples)

    def __iter__(self):
        return self

    def __next__(self):
        if self._counter == self._num_updates:
            raise StopIteration
        if self._pool.size < self._batch_size:  # a fresh shuffled epoch
            self._pool = self._rng.permutation(self._n_samples)
        batch, self._pool = self._pool[: self._batch_size], self._pool[self._batch_size :]
        self._counter += 1
        return batch

    def reset_counter(self):
        self._counter = 0

    def check_num_updates(self):
        if self._counter != self._num_updates:
            raise IndexGeneratorUpdateError(f"drawn {self._counter} batches, expected {self._num_updates}")
