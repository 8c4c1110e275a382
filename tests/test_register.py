"""ROCm base image for docker/remote mode (substrafl_amd.remote.register; register.py:49-62,144-162)."""

import pytest

from substrafl_amd.remote import register


def test_rocm_gpu_image():
    img = register.get_base_docker_image("3.12", use_gpu=True, custom_binary_dependencies=["libgl1"])
    assert "FROM rocm/dev-ubuntu-24.04:7.2" in img
    assert "python3.12 python3.12-venv" in img and "libgl1" in img
    assert "deadsnakes" not in img and "nvidia" not in img
    # what the substrafl_amd build hook needs in the image (setup.py -> __graft_entry__._hipcc)
    assert "HIPCC=/opt/rocm/bin/hipcc" in img and "PATH=/opt/rocm/bin:$PATH" in img
    img10 = register.get_base_docker_image("3.10", use_gpu=True)
    assert "deadsnakes" in img10 and "python3.10-venv" in img10


def test_cpu_images_and_versions():
    assert "FROM python:3.11-slim" in register.get_base_docker_image("3.11", use_gpu=False)
    assert "apt-get install -y git" in register.get_base_docker_image("3.11", False, ["git"])
    for bad in ("3.9", "3.13", "2.7"):
        with pytest.raises(register.UnsupportedPythonVersionError):
            register.get_base_docker_image(bad, use_gpu=True)
    with pytest.raises(ValueError):
        register.get_base_docker_image("3.12", use_gpu=True, gpu_vendor="nvidia")
