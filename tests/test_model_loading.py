"""The aggregation outputs load back through the reference's model-loading path
(model_loading.py:240-283, offline part) without touching the GPU."""

import json
import pickle
import tarfile

import numpy as np
import pytest

from substrafl_amd import model_loading, runtime, wire
from substrafl_amd.exceptions import LoadFileNotFoundError, LoadMetadataError
from substrafl_amd.remote import RemoteStruct
from substrafl_amd.remote.substratools_methods import RemoteMethod
from substrafl_amd.schemas import FedAvgAveragedState
from substrafl_amd.strategies import FedAvg


def _folder(tmp_path, dummy_algo_class, state):
    internal = tmp_path / "build" / model_loading.SUBSTRAFL_FOLDER
    internal.mkdir(parents=True)
    RemoteStruct(FedAvg, [], {"algo": dummy_algo_class()}, RemoteMethod, "avg_shared_states", {}, None).save(internal)
    out = tmp_path / "out"
    out.mkdir()
    with tarfile.open(out / "function.tar.gz", "w:gz") as tar:
        tar.add(internal, arcname=model_loading.SUBSTRAFL_FOLDER)
    with open(out / "model", "wb") as f:
        pickle.dump(state, f)
    (out / "metadata.json").write_text(json.dumps({"model_file": "model", "function_file": "function.tar.gz"}))
    return out


@pytest.mark.parametrize("flat", [False, True])
def test_aggregate_state_loads_back(tmp_path, dummy_algo_class, flat):
    rng = np.random.default_rng(0)
    layers = [rng.standard_normal(s).astype(np.float32) for s in [(3, 4), (4,), (1,)]]
    avg = wire.pack(layers) if flat else layers
    folder = _folder(tmp_path, dummy_algo_class, FedAvgAveragedState(avg_parameters_update=avg))
    warming = dict(runtime._warming)
    got = model_loading.load_from_files(folder, remote=True)
    assert isinstance(got, FedAvgAveragedState)
    for g, r in zip(got.avg_parameters_update, layers):
        assert isinstance(g, np.ndarray) and g.dtype == r.dtype and np.array_equal(g, r)
    assert runtime._warming == warming  # loading a model never starts the GPU runtime


def test_folder_validation(tmp_path):
    with pytest.raises(LoadFileNotFoundError):
        model_loading.load_from_files(tmp_path)
    (tmp_path / "metadata.json").write_text(json.dumps({"function_file": "f"}))
    with pytest.raises(LoadMetadataError):
        model_loading.load_from_files(tmp_path)
    (tmp_path / "metadata.json").write_text(json.dumps({"function_file": "f", "model_file": "m"}))
    with pytest.raises(LoadFileNotFoundError, match="m, f"):
        model_loading.load_from_files(tmp_path)
