"""Wheel build: compiles the native extensions in-tree before packaging them.

The reference ships maturin wheels of its Rust core (.github/workflows/publish-pypi.yml).
Here ``build_py`` first runs ``relayrl_prototype_amd/_build.py``. That compiles the
gfx950 HIP kernels and the C++ host runtime. The resulting ``_hip_ops*.so`` and
``_native*.so`` then travel as package data.

    RRL_BUILD_TARGETS=native pip wheel . --no-deps --no-build-isolation   # host runtime only
    pip wheel . --no-deps --no-build-isolation                            # + HIP kernels (hipcc)
"""
import importlib.util
import os

from setuptools import Distribution, find_packages, setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))


class BuildWithNative(build_py):
    def run(self):
        # Load _build.py by path: importing the package would pull in torch-dependent modules.
        spec = importlib.util.spec_from_file_location(
            "_rrl_build", os.path.join(HERE, "relayrl_prototype_amd", "_build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        targets = tuple(t for t in os.environ.get("RRL_BUILD_TARGETS", "native,hip").split(",") if t)
        mod.build(targets, verbose=bool(os.environ.get("RRL_BUILD_VERBOSE")))
        super().run()


class BinaryDistribution(Distribution):
    """The wheel carries compiled .so files, so it is platform-specific."""

    def has_ext_modules(self):
        return True


setup(
    name="relayrl-prototype-amd",
    version="0.1.0",
    description="MI355X-native (gfx950) actor-learner RL engine with the RelayRL-prototype API",
    long_description=open(os.path.join(HERE, "README.md")).read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.9",
    packages=find_packages(include=["relayrl_prototype_amd*", "relayrl_framework*"]),
    package_data={"relayrl_prototype_amd": ["*.so"]},
    install_requires=["torch>=2.5", "numpy", "pyyaml"],
    extras_require={"grpc": ["grpcio", "protobuf"], "logging": ["pandas"],
                    "test": ["pytest", "hypothesis", "pytest-timeout"]},
    entry_points={"console_scripts": ["relayrl = relayrl_prototype_amd.runtime.launcher:main"]},
    cmdclass={"build_py": BuildWithNative},
    distclass=BinaryDistribution,
)
