"""pytest plugin (CONTAINER-ONLY checker, loaded with ``-p fedagg_refstubs`` by
tests/reference_own_tests.py): the import stubs for the absent ``substra`` / ``substratools`` /
``docker`` packages that the reference's own test suite imports at module level (the same
permissive stubs as tests/golden/gen_golden.py), so its strategy unit tests can run in place."""

import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "golden"))
from gen_golden import _install_stubs  # noqa: E402

_install_stubs()
sys.modules["substra"].BackendType = types.SimpleNamespace(REMOTE="remote", LOCAL_SUBPROCESS="subprocess",
                                                           LOCAL_DOCKER="docker")
