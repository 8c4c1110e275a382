"""FedAvg's client: apply the averaged update, train, return the weight delta and put the
weights back (the reference's ``TorchFedAvgAlgo.train`` sequence), in per-layer torch ops."""

import torch

from ...remote import remote_data
from ...strategies.schemas import FedAvgSharedState, StrategyName
from . import _weights as w
from .torch_base_algo import TorchAlgo


class TorchFedAvgAlgo(TorchAlgo):
    def __init__(self, model, criterion, optimizer, index_generator, dataset, scheduler=None,
                 with_batch_norm_parameters: bool = False, disable_gpu: bool = False, *args, **kwargs):
        super().__init__(model, criterion, index_generator, dataset, optimizer, scheduler, disable_gpu,
                         *args, **kwargs)
        self._with_batch_norm_parameters = with_batch_norm_parameters

    @property
    def strategies(self):
        return [StrategyName.FEDERATED_AVERAGING]

    @remote_data
    def train(self, data_from_opener, shared_state=None):
        bn = self._with_batch_norm_parameters
        ds = self._dataset(data_from_opener, is_inference=False)
        if shared_state is None:
            assert self._index_generator.n_samples is None
            self._index_generator.n_samples = len(ds)
        else:
            assert self._index_generator.n_samples is not None
            w.add_into(self._model, [torch.from_numpy(a).to(self._device) for a in shared_state.avg_parameters_update],
                       bn)
        self._index_generator.reset_counter()
        start = w.snapshot(self._model, bn)
        self._model.train()
        self._local_train(ds)
        self._index_generator.check_num_updates()
        self._model.eval()
        delta = w.combine([w.snapshot(self._model, bn), start], [1, -1])
        w.rebind(self._model, start, bn)
        return FedAvgSharedState(n_samples=len(ds), parameters_update=[t.cpu().detach().numpy() for t in delta])
