"""CONTAINER-ONLY checker (imports /root/reference; never runs on the GPU box): the reference's own
dependency machinery ships ``substrafl_amd`` to a task image (VERDICT r04 "Next 2").

``substrafl.dependency.Dependency(local_installable_dependencies=[<repo>])`` validates the
directory (schemas.py:109-124: a ``setup.py`` or ``pyproject.toml`` must be there), copies it
(path_management.copy_paths, with the caller's ``excluded_paths``) and builds its wheel with
``pip wheel <copy>/ --no-deps`` (manage_dependencies.py:24-58), whose build hook (setup.py)
compiles ``libfedagg.so`` for gfx950 into it.  That wheel is what the task image's
``requirements.txt`` installs (register.py:60-110).  The container has no package index, so pip
runs without build isolation (``PIP_NO_BUILD_ISOLATION=0``, the image's setuptools); a user's
machine with an index builds the same wheel in isolation.  Prints one JSON line.
"""

from __future__ import annotations

import json
import os
import sys
import zipfile
from pathlib import Path

sys.dont_write_bytecode = True  # never write into /root/reference
HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
sys.path.insert(0, str(HERE / "golden"))
from gen_golden import REF, _install_stubs  # noqa: E402

# what a maintainer excludes when shipping the repo as a task dependency
EXCLUDED = [".git", "gpurun_out", "profiles", "tests", "tools", "scripts", "oracle", "build",
            "substrafl_amd/libfedagg_tuning.so"]


def main():
    if not REF.exists():
        raise SystemExit("reference_dependency.py needs /root/reference (build container only)")
    os.environ.update(PIP_NO_BUILD_ISOLATION="0", PIP_NO_INDEX="1")
    _install_stubs()
    sys.path.insert(0, str(REF))
    from substrafl import exceptions
    from substrafl.dependency import Dependency

    out = {}
    dep = Dependency(local_installable_dependencies=[ROOT], excluded_paths=[ROOT / p for p in EXCLUDED])
    wheels = [Path(w) for w in dep._wheels]
    out["wheels"] = [w.name for w in wheels]
    whl = dep.cache_directory / wheels[0]
    names = zipfile.ZipFile(whl).namelist()
    out["wheel_has_library"] = any(n.endswith("substrafl_amd/libfedagg.so") for n in names)
    out["wheel_has_package"] = any(n.endswith("substrafl_amd/strategies/fed_avg.py") for n in names)
    out["wheel_has_tests"] = any("/tests/" in n or n.startswith("tests/") for n in names)
    req = (dep.cache_directory / "requirements.txt").read_text()
    out["requirements_name_the_wheel"] = wheels[0].name in req

    # the validator still refuses a directory that is not an installable package
    try:
        Dependency(local_installable_dependencies=[ROOT / "include"])
        out["non_package_dir"] = "accepted"
    except exceptions.InvalidPathError:
        out["non_package_dir"] = "InvalidPathError"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
