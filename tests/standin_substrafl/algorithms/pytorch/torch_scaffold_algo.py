"""Scaffold's client (the reference's ``TorchScaffoldAlgo.train`` sequence, option II control
variate rule): per-step ``w += lr * (c_i - c)``, weight delta, ``c_i`` update, in per-layer torch
ops."""

from enum import IntEnum

import torch

from ...exceptions import TorchScaffoldAlgoParametersUpdateError
from ...remote import remote_data
from ...strategies.schemas import ScaffoldSharedState, StrategyName
from . import _weights as w
from .torch_base_algo import TorchAlgo


class CUpdateRule(IntEnum):
    STABLE = 1
    FAST = 2


class TorchScaffoldAlgo(TorchAlgo):
    def __init__(self, model, criterion, optimizer, index_generator, dataset, scheduler=None,
                 with_batch_norm_parameters: bool = False, c_update_rule=CUpdateRule.FAST,
                 disable_gpu: bool = False, *args, **kwargs):
        super().__init__(model, criterion, index_generator, dataset, optimizer, scheduler, disable_gpu,
                         *args, **kwargs)
        self._with_batch_norm_parameters = with_batch_norm_parameters
        self._c_update_rule = CUpdateRule(c_update_rule)
        self._client_control_variate = None
        self._server_control_variate = None
        self._delta_variate = None
        self._current_lr = None
        self._scaffold_parameters_update_num_call = 0

    @property
    def strategies(self):
        return [StrategyName.SCAFFOLD]

    def _update_current_lr(self):
        lrs = {g["lr"] for g in self._optimizer.param_groups} - {0}
        self._current_lr = float(min(lrs))

    def _scaffold_parameters_update(self):
        self._update_current_lr()
        self._scaffold_parameters_update_num_call += 1
        w.add_into(self._model, self._delta_variate, self._with_batch_norm_parameters, self._current_lr)

    def _reset_scaffold_parameters_update(self):
        self._scaffold_parameters_update_num_call = 0

    def _step_hook(self):
        self._scaffold_parameters_update()

    @remote_data
    def train(self, data_from_opener, shared_state=None):
        bn = self._with_batch_norm_parameters
        ds = self._dataset(data_from_opener, is_inference=False)
        gen = self._index_generator
        if shared_state is None:
            assert gen.n_samples is None
            gen.n_samples = len(ds)
            assert self._client_control_variate is None and self._server_control_variate is None
            self._client_control_variate = w.zeros(self.model, bn, self._device)
            self._server_control_variate = w.zeros(self.model, bn, self._device)
        else:
            assert self._client_control_variate is not None and gen.n_samples is not None
            w.add_into(self._model, [torch.from_numpy(a).to(self._device) for a in shared_state.avg_parameters_update],
                       bn)
            self._server_control_variate = [torch.from_numpy(a).to(self._device)
                                            for a in shared_state.server_control_variate]
        gen.reset_counter()
        start = w.snapshot(self._model, bn)
        self._delta_variate = w.combine([self._client_control_variate, self._server_control_variate], [1, -1])
        self._model.train()
        self._local_train(ds)
        gen.check_num_updates()
        if self._scaffold_parameters_update_num_call != gen._num_updates:
            raise TorchScaffoldAlgoParametersUpdateError("the Scaffold hook must run once per update")
        self._reset_scaffold_parameters_update()
        self._model.eval()
        delta = w.combine([w.snapshot(self._model, bn), start], [1, -1])
        if self._c_update_rule != CUpdateRule.FAST:
            raise NotImplementedError("rule 1 not implemented")
        cv_update = w.combine([self._server_control_variate, delta], [-1.0, -1.0 / (self._current_lr * gen.num_updates)])
        self._client_control_variate = w.combine([self._client_control_variate, cv_update], [1, 1])
        w.rebind(self._model, start, bn)
        host = lambda ts: [t.cpu().detach().numpy() for t in ts]  # noqa: E731
        return ScaffoldSharedState(parameters_update=host(delta), control_variate_update=host(cv_update),
                                   server_control_variate=host(self._server_control_variate), n_samples=len(ds))
