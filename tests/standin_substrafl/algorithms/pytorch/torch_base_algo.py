"""The torch algorithm base: model on the device, the default training loop over the index
generator's batches (the reference's ``TorchAlgo`` contract: ``args`` / ``kwargs`` kept for the
re-creation of the class, ``_device`` = the GPU unless disabled), written for this stand-in."""

import torch


class TorchAlgo:
    def __init__(self, model, criterion, index_generator, dataset, optimizer=None, scheduler=None,
                 disable_gpu: bool = False, *args, **kwargs):
        self.args, self.kwargs = args, kwargs
        self.disable_gpu = disable_gpu
        self._model = model.to(self._device)
        self._criterion = criterion
        self._optimizer = optimizer
        self._scheduler = scheduler
        self._index_generator = index_generator
        self._dataset = dataset

    @property
    def model(self):
        return self._model

    @property
    def _device(self):
        return torch.device("cuda" if torch.cuda.is_available() and not self.disable_gpu else "cpu")

    def _step_hook(self):
        """Called after every optimizer step (Scaffold adds its control-variate term here)."""

    def _local_train(self, train_dataset):
        loader = torch.utils.data.DataLoader(train_dataset, batch_sampler=self._index_generator)
        for xb, yb in loader:
            xb, yb = xb.to(self._device), yb.to(self._device)
            loss = self._criterion(self._model(xb), yb)
            self._optimizer.zero_grad()
            loss.backward()
            self._optimizer.step()
            self._step_hook()
            if self._scheduler is not None:
                self._scheduler.step()
