"""Loading an aggregated shared state from a downloaded task-output folder (egress of the hot
path; SURVEY.md §3.5, north_star's model_loading.py).

The reference's ``download_aggregate_shared_state`` (``substrafl/model_loading.py:447-478``) downloads
a task's output files with a Substra client and calls ``_load_from_files(folder, remote=True)``
(``:240-283``): check ``metadata.json`` (``:64-114``), extract ``function.tar.gz`` and re-create the
remote instance from its ``RemoteStruct`` (``:152-178``), then ``instance.load_shared(model_file)``.
The download needs the Substra backend (out of scope); this module is the offline part, so the
engine's outputs (plain arrays, or the flat wire format of :mod:`substrafl_amd.wire`) are proven to
load back the way the reference loads them.  Loading never starts the GPU: the remote instance is
built but its function is not registered (see ``RemoteMethod.register_substratools_function``).
"""

from __future__ import annotations

import json
import tarfile
from pathlib import Path
from typing import Any

from .exceptions import LoadFileNotFoundError, LoadMetadataError
from .remote.remote_struct import RemoteStruct

SUBSTRAFL_FOLDER = "substrafl_internal"  # constants.py:2
METADATA_FILE = "metadata.json"
FUNCTION_DICT_KEY = "function_file"
MODEL_DICT_KEY = "model_file"


def validate_folder_content(folder: Path) -> dict:
    """model_loading.py:64-114: metadata.json present, naming an existing model and function file."""
    folder = Path(folder)
    meta_path = folder / METADATA_FILE
    if not meta_path.exists():
        raise LoadFileNotFoundError(f"{METADATA_FILE} not found within the provided input folder `{folder}`.")
    metadata = json.loads(meta_path.read_text())
    for key in (MODEL_DICT_KEY, FUNCTION_DICT_KEY):
        if key not in metadata:
            raise LoadMetadataError(f"The {METADATA_FILE} file from the specified folder should contain a `{key}` key.")
    missing = [metadata[k] for k in (MODEL_DICT_KEY, FUNCTION_DICT_KEY) if not (folder / metadata[k]).exists()]
    if missing:
        raise LoadFileNotFoundError(", ".join(missing) + f" not found within the provided input folder `{folder}`.")
    return metadata


def load_instance(gz_path: Path, extraction_folder: Path, remote: bool) -> Any:
    """model_loading.py:152-178: extract the function archive, re-create the (remote) instance."""
    with tarfile.open(gz_path, "r:gz") as tar:
        if hasattr(tarfile, "data_filter"):
            tar.extractall(path=extraction_folder, filter="data")
        else:  # pragma: no cover - Python without PEP 706
            tar.extractall(path=extraction_folder)
    struct = RemoteStruct.load(Path(extraction_folder) / SUBSTRAFL_FOLDER)
    return struct.get_remote_instance() if remote else struct.get_instance()


def load_from_files(input_folder: Path, remote: bool = True) -> Any:
    """model_loading.py:240-283 (``remote=True``: a shared / aggregated state)."""
    folder = Path(input_folder)
    metadata = validate_folder_content(folder)
    instance = load_instance(folder / metadata[FUNCTION_DICT_KEY], folder, remote)
    if remote:
        return instance.load_shared(folder / metadata[MODEL_DICT_KEY])
    return instance.load_local_state(folder / metadata[MODEL_DICT_KEY])
