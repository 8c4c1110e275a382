"""ROCm base image for Substra's docker / remote execution modes.

The reference picks the task image in ``_get_base_docker_image``
(``substrafl/remote/register/register.py:144-162``); with ``Dependency(use_gpu=True)`` it is a
CUDA runtime image (``:49-60``), on which ``libfedagg.so`` cannot run.  This module provides the
same function with a ROCm branch: the HIP runtime image of the ROCm release the library is built
against, Python from the distribution (or deadsnakes for other minor versions), and the system
packages the caller lists.  ``INTEGRATION.md`` shows where a maintainer plugs it in.

Only the base-image text is produced here; the rest of the Dockerfile (non-root user, venv,
requirements, entrypoint) stays the reference's template.  The aggregation task does not need
PyTorch in the image: the drop-in path runs on ``libfedagg.so``'s native session alone.
At run time the container needs the ROCm devices (``--device /dev/kfd --device /dev/dri``) and
its user in their groups (``--group-add video --group-add render``), which is the backend's
``docker run`` configuration, not the image's.
"""

from __future__ import annotations

from typing import Optional, Sequence

ROCM_VERSION = "7.2"  # the release libfedagg.so is compiled and tested with (gfx950)
UBUNTU = "24.04"
_UBUNTU_PYTHON = {"24.04": "3.12", "22.04": "3.10"}

MINIMAL_PYTHON_MINOR = 10  # register.py:27-29 (3.10 .. 3.12)
MAXIMAL_PYTHON_MINOR = 12


class UnsupportedPythonVersionError(Exception):
    """Same meaning as ``substrafl.exceptions.UnsupportedPythonVersionError``."""


def check_python_version(python_major_minor: str) -> None:
    """register.py:131-141: only 3.10 to 3.12 are supported."""
    major, minor = python_major_minor.split(".")
    if major != "3":
        raise UnsupportedPythonVersionError("Only Python 3 is supported")
    if not MINIMAL_PYTHON_MINOR <= int(minor) <= MAXIMAL_PYTHON_MINOR:
        raise UnsupportedPythonVersionError(
            f"The current Python version is {python_major_minor}, which is unsupported; "
            f"supported versions are 3.{MINIMAL_PYTHON_MINOR} to 3.{MAXIMAL_PYTHON_MINOR}"
        )


def rocm_base_image(python_major_minor: str, binary_dependencies: Optional[Sequence[str]] = None,
                    rocm_version: str = ROCM_VERSION, ubuntu: str = UBUNTU) -> str:
    """Dockerfile lines of a ROCm HIP-runtime base with ``python{python_major_minor}`` installed."""
    check_python_version(python_major_minor)
    extra = " ".join(binary_dependencies or [])
    py = f"python{python_major_minor}"
    if _UBUNTU_PYTHON.get(ubuntu) == python_major_minor:
        install_python = f"apt-get install -y --no-install-recommends {py} {py}-venv python3-pip {extra}"
    else:
        install_python = ("apt-get install -y --no-install-recommends software-properties-common"
                          " && add-apt-repository -y ppa:deadsnakes/ppa && apt-get update -y"
                          f" && apt-get install -y --no-install-recommends {py} {py}-venv python3-pip {extra}")
    return (
        f"\nFROM rocm/dev-ubuntu-{ubuntu}:{rocm_version}\n\n"
        "# HIP runtime for libfedagg.so (gfx950); Python for the task entrypoint.  The substrafl_amd\n"
        "# wheel carries the compiled library; hipcc stays on PATH so a source install builds it too\n"
        "ENV DEBIAN_FRONTEND=noninteractive HSA_ENABLE_IPC_MODE_LEGACY=0 HIPCC=/opt/rocm/bin/hipcc \\\n"
        "    PATH=/opt/rocm/bin:$PATH LD_LIBRARY_PATH=/opt/rocm/lib\n"
        f"RUN apt-get update -y && {install_python.strip()}"
        " && apt-get clean && rm -rf /var/lib/apt/lists/*\n\n"
    )


def get_base_docker_image(python_major_minor: str, use_gpu: bool,
                          custom_binary_dependencies: Optional[list] = None, gpu_vendor: str = "amd") -> str:
    """register.py:144-162 with a ROCm GPU branch.  ``gpu_vendor="nvidia"`` is not provided here:
    a maintainer keeps the reference's own CUDA branch for it."""
    if use_gpu:
        if gpu_vendor != "amd":
            raise ValueError("only the ROCm (gpu_vendor='amd') GPU image is provided by substrafl_amd")
        return rocm_base_image(python_major_minor, custom_binary_dependencies)
    check_python_version(python_major_minor)
    lines = [f"\nFROM python:{python_major_minor}-slim\n", "RUN apt-get update -y && pip uninstall -y setuptools"]
    if custom_binary_dependencies:
        lines[-1] += " && apt-get install -y " + " ".join(custom_binary_dependencies) + " && apt-get clean"
    return "\n".join(lines) + "\n"
