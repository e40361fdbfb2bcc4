"""Packaging for ray_lightning_accelerators_amd (MI355X / gfx950).

``pip install .`` (or ``python setup.py build_ext --inplace``) compiles the HIP
extensions with hipcc for gfx950 through ``ray_lightning_accelerators_amd._build``
and places ``_C`` / ``_comm`` next to the Python sources.  The reference's
``setup.py`` only declared ``pytorch-lightning`` and ``ray``; this package carries
its own Lightning / Ray / Tune / Horovod subsets, so its runtime dependency is
PyTorch-ROCm (plus cloudpickle, numpy).
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class HipBuildExt(build_ext):
    """Builds every HIP extension in-tree (gfx950), then copies it into build_lib."""

    def run(self):
        sys.path.insert(0, ROOT)
        from ray_lightning_accelerators_amd import _build

        built = _build.build_all(force=self.force, jobs=int(os.environ.get("MAX_JOBS", "8")), verbose=True)
        if not self.inplace:
            dst = os.path.join(self.build_lib, "ray_lightning_accelerators_amd")
            os.makedirs(dst, exist_ok=True)
            for p in built:
                self.copy_file(str(p), os.path.join(dst, os.path.basename(str(p))))


class BuildPyWithExt(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(
    name="ray_lightning_accelerators_amd",
    version="0.1.0",
    description="MI355X-native distributed Lightning training (RayAccelerator / HorovodRayAccelerator API)",
    packages=find_packages(include=["ray_lightning_accelerators_amd*", "ray_lightning*"]),
    package_data={"ray_lightning_accelerators_amd": ["csrc/*.h", "csrc/*.hip", "csrc/*.cpp", "csrc/comm/*"]},
    python_requires=">=3.8",
    install_requires=["torch", "cloudpickle", "numpy"],
    cmdclass={"build_ext": HipBuildExt, "build_py": BuildPyWithExt},
    zip_safe=False,
)
