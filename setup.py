"""Build hook of the installable package (pyproject.toml): ``build_py`` also compiles
``libfedagg.so`` for gfx950 into the build tree with the same compiler, flags and object cache as
``__graft_entry__.build()``, so the wheel carries the HIP library next to the Python package.
No hipcc, no wheel: ``compile_library`` raises, and the build fails loudly."""

import sys
from pathlib import Path

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

ROOT = Path(__file__).resolve().parent


class BuildPyWithHip(build_py):
    def run(self):
        super().run()
        sys.path.insert(0, str(ROOT))
        import __graft_entry__

        __graft_entry__.compile_library(Path(self.build_lib).resolve() / "substrafl_amd" / "libfedagg.so")


class BinaryDistribution(Distribution):
    """The wheel holds a gfx950 shared library: a platform wheel, never ``py3-none-any``."""

    def has_ext_modules(self):
        return True


setup(
    packages=find_packages(include=["substrafl_amd", "substrafl_amd.*"]),
    package_data={"substrafl_amd": ["csrc/*.hip", "csrc/*.h"]},
    cmdclass={"build_py": BuildPyWithHip},
    distclass=BinaryDistribution,
    zip_safe=False,
)
