"""Packaging for grace_amd (the reference ships a pure distutils setup.py: setup.py:1-10).

The native extension is built IN-TREE by grace_amd/_build.py (hipcc --offload-arch=gfx950,
linked against the installed PyTorch-ROCm and RCCL) before the package files are collected:

    python setup.py build_ext        # or: python -m grace_amd._build
    pip install --no-build-isolation --no-deps -e .
"""
from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext
from setuptools.command.build_py import build_py


class _BuildHip(build_ext):
    def run(self):
        from grace_amd import _build

        _build.build()


class _BuildPy(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(
    name="grace_amd",
    version="0.1.0",
    description="MI355X-native GRACE gradient compression (HIP/CDNA4 kernels, RCCL over xGMI)",
    packages=find_packages(include=["grace_amd", "grace_amd.*"]),
    package_data={"grace_amd": ["_C.so"]},
    python_requires=">=3.10",
    install_requires=["torch"],
    cmdclass={"build_ext": _BuildHip, "build_py": _BuildPy},
)
